"""The Go EnricherInterface adapter's flow -> record inverse (go/pkg/gpuagg/enricher_linux.go
flowToRecord; there is no Go toolchain in the image, so its mapping is transcribed here
statement by statement and checked): a record the producers' ToFlow / AddTCPFlags /
AddDropReason / AddDNSInfo turn into a flow (oracle.records.flow_from_record restates
them, flow_utils.go:33-300) and the adapter turns back must give every metric series the
original gives -- in the oracle and through the engine's CPU backend -- so unmodified
producers feeding the engine through Write(*v1.Event) get the reference's series."""

import zlib

import pytest

from oracle import oracle as O
from oracle import records as R
from retina_amd import workloads as W

from .helpers import diff_series, dns_dict, engine_series, oracle_series
from .test_gpu_parity import CASES

_OBS = {O.OBS_TO_ENDPOINT: 1, O.OBS_FROM_NETWORK: 2, O.OBS_TO_NETWORK: 3}


def go_flow_to_record(f: O.Flow, intern):
    """enricher_linux.go flowToRecord, line for line (None: dropped like enrich does)."""
    ip = f.ip
    if ip is None or ip.ip_version > 1 or ip.source == "" or ip.destination == "":
        return None
    src, dst = O.ip2int(ip.source), O.ip2int(ip.destination)
    proto = sport = dport = flags = 0
    if f.l4 is not None and f.l4.proto == "TCP":
        proto, sport, dport = 6, f.l4.source_port, f.l4.destination_port
        fl = f.l4.flags
        if fl is not None:
            flags = int(fl.FIN) | int(fl.SYN) << 1 | int(fl.RST) << 2 | int(fl.PSH) << 3 | int(fl.ACK) << 4 | \
                int(fl.URG) << 5
    elif f.l4 is not None and f.l4.proto == "UDP":
        proto, sport, dport = 17, f.l4.source_port, f.l4.destination_port
    meta = f.extensions if f.extensions is not None else O.RetinaMetadata()
    obs = _OBS.get(f.trace_observation_point, 0)
    verdict = f.verdict & 0xFF
    m = (proto | verdict << 8 | (f.traffic_direction & 3) << 16 | (meta.drop_reason & 7) << 18 | flags << 21 |
         int(bool(f.is_reply)) << 27 | (meta.dns_type & 3) << 28 | obs << 30)
    dns_id = 0xFFFFFFFF
    if f.dns is not None:
        dns_id = intern(f.dns.rcode, tuple(f.dns.qtypes), f.dns.query, tuple(f.dns.ips), meta.num_responses)
    return (src, dst, meta.bytes, m, sport | dport << 16, dns_id, meta.tcp_id & 0xFFFFFFFF, f.time_ns)


def _round_trip(recs):
    """records -> producer flows -> adapter records, with the adapter's own DNS ids."""
    dd = dns_dict(recs)
    ids, payload = {}, []

    def intern(rcode, qtypes, query, ips, n):
        key = (rcode, qtypes, query, ips, n)
        if key not in ids:
            ids[key] = len(payload)
            payload.append(R.DnsEntry(rcode, list(qtypes), query, list(ips), n))
        return ids[key]
    rows = []
    for i in range(len(recs.src_ip)):
        f = R.flow_from_record(int(recs.src_ip[i]), int(recs.dst_ip[i]), int(recs.bytes[i]), int(recs.meta[i]),
                               int(recs.ports[i]), int(recs.dns_id[i]), dd)
        r = go_flow_to_record(f, intern)
        assert r is not None
        rows.append(r)
    import numpy as np
    cols = [np.array([r[k] for r in rows], np.uint32) for k in range(6)]
    dns = [W.DnsPayload(p.rcode, p.qtypes, p.query, p.ips, p.num_answers) for p in payload]
    return W.Records(*cols, dns)


@pytest.mark.parametrize("cid,sp,remote,gen", CASES, ids=[c[0] for c in CASES])
def test_adapter_round_trip_keeps_every_series(cid, sp, remote, gen):
    pods = W.make_pods(200, seed=17)
    recs = W.gen_records(4_000, pods, seed=zlib.crc32(cid.encode()) & 0xFFFF, **gen)
    back = _round_trip(recs)
    want = oracle_series(recs, pods, sp, remote)
    assert oracle_series(back, pods, sp, remote) == want
    got = engine_series(back, pods, sp, remote, host_fed=True, flags=128)  # CPU backend
    assert got == want, diff_series(got, want)


def test_adapter_drops_what_enrich_drops():
    f = O.to_flow("10.0.0.1", "10.0.0.2", 1, 2, 6, 3, 1)
    f.ip.ip_version = 2  # IPv6: enricher.go:107-110 returns before export
    assert go_flow_to_record(f, None) is None
    f = O.to_flow("10.0.0.1", "10.0.0.2", 1, 2, 6, 3, 1)
    f.ip.destination = ""  # enricher.go:121-124
    assert go_flow_to_record(f, None) is None
