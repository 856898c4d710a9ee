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
    if f.traffic_direction > 3 or (f.verdict == O.VERDICT_DROPPED and meta.drop_reason > 7):
        verdict = 255  # what the raw decode leaves out too (PacketRecord / DropRecord)
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


# ---- go/pkg/gpuagg/gpuagg_linux.go helpers, transcribed ------------------------------

def go_ipv4_le(s: str):
    """gpuagg_linux.go ipv4LE, line for line: the allocation-free dotted-quad path, else
    ('slow', s) -- the net.ParseIP fallback."""
    v = oct_ = digits = dots = 0
    for ch in s:
        if "0" <= ch <= "9":
            if digits > 0 and oct_ == 0:
                return ("slow", s)
            oct_ = oct_ * 10 + (ord(ch) - 48)
            digits += 1
            if digits > 3 or oct_ > 255:
                return ("slow", s)
        elif ch == ".":
            if digits == 0 or dots == 3:
                return ("slow", s)
            v |= oct_ << (8 * dots)
            dots += 1
            oct_ = digits = 0
        else:
            return ("slow", s)
    if dots != 3 or digits == 0:
        return ("slow", s)
    return v | oct_ << 24


def _parse_ip_to4(s: str):
    """net.ParseIP(s).To4() read little-endian (Go >= 1.17: IPv4 octets with leading zeros
    rejected; IPv4-mapped IPv6 text gives its IPv4).  Python's ipaddress has the same
    IPv4 rules (3.9.5+)."""
    import ipaddress
    try:
        a = ipaddress.ip_address(s)
    except ValueError:
        return None
    if a.version == 6:
        a = a.ipv4_mapped
        if a is None:
            return None
    return int.from_bytes(a.packed, "little")


def test_ipv4le_fast_path_is_parseip():
    import random
    rng = random.Random(7)
    cases = ["0.0.0.0", "255.255.255.255", "10.0.0.1", "1.2.3.4", "01.2.3.4", "1.2.3.04", "1.2.3", "1.2.3.4.5",
             "256.1.1.1", "1..2.3", ".1.2.3", "1.2.3.", "", "a.b.c.d", "1.2.3.4 ", "::ffff:10.1.2.3", "::1",
             "1000.1.1.1", "00.0.0.0", "0.00.0.0", "192.168.001.1", "-1.2.3.4", "1.2.3.+4"]
    for _ in range(3000):
        parts = [str(rng.choice([rng.randrange(256), rng.randrange(1000), 0])) for _ in range(rng.choice([3, 4, 4, 5]))]
        if rng.random() < 0.1:
            i = rng.randrange(len(parts))
            parts[i] = "0" + parts[i]
        cases.append(".".join(parts))
    fast = 0
    for s in cases:
        want = _parse_ip_to4(s)
        got = go_ipv4_le(s)
        if isinstance(got, tuple):
            got = _parse_ip_to4(got[1])  # the fallback is net.ParseIP itself
        else:
            fast += 1
            assert want is not None, s  # the fast path never accepts what ParseIP rejects
        assert got == want, s
        if want is not None and ":" not in s:
            assert not isinstance(go_ipv4_le(s), tuple), s  # every dotted quad takes the fast path
    assert fast > 300


def go_packet_record(r):
    """gpuagg_linux.go PacketRecord on the fields of one struct packet (time offset 0)."""
    swap = lambda x: ((x & 0xFF) << 8) | (x >> 8)  # bits.ReverseBytes16
    verdict = 255 if r["tdir"] > 3 else 1
    tcp_flags = int(r["flags"]) & 0x3F if r["proto"] == 6 else 0
    obs = int(r["obs"]) if r["obs"] <= 3 else 0
    meta = (int(r["proto"]) | verdict << 8 | (int(r["tdir"]) & 3) << 16 | tcp_flags << 21 |
            int(bool(r["is_reply"])) << 27 | obs << 30)
    tcp_id = int(r["tsval"]) if r["obs"] == 3 else int(r["tsecr"]) if r["obs"] == 2 else 0
    return (int(r["src_ip"]), int(r["dst_ip"]), int(r["bytes"]), meta,
            swap(int(r["src_port"])) | swap(int(r["dst_port"])) << 16, 0xFFFFFFFF, tcp_id, int(r["t_nsec"]))


def go_drop_record(r):
    """gpuagg_linux.go DropRecord on the fields of one dropreason struct packet."""
    swap = lambda x: ((x & 0xFF) << 8) | (x >> 8)
    verdict = 255 if r["drop_type"] > 7 else 2
    meta = int(r["proto"]) | verdict << 8 | 1 << 16 | (int(r["drop_type"]) & 7) << 18 | 2 << 30
    return (int(r["src_ip"]), int(r["dst_ip"]), int(r["skb_len"]), meta,
            swap(int(r["src_port"])) | swap(int(r["dst_port"])) << 16, 0xFFFFFFFF, 0, int(r["ts"]))


@pytest.mark.parametrize("kind", ["packet", "drop"])
def test_record_constructors_equal_the_decode(kind):
    """PacketRecord / DropRecord (the INTEGRATION.md producer snippets) give the columns the
    raw decode gives (oracle/decode.py, pinned to the per-record oracle)."""
    import numpy as np
    from oracle import decode as D
    pods = W.make_pods(100, seed=3)
    if kind == "packet":
        raw = W.gen_raw_packets(3000, pods, seed=11, odd_frac=0.3, out_of_range_frac=0.05)
        batch, _ = D.decode_packets(raw)
        rows = np.frombuffer(raw.tobytes(), D.PACKET_DTYPE)
        conv = go_packet_record
    else:
        raw = W.gen_raw_drops(3000, pods, seed=12, out_of_range_frac=0.05)
        batch, _ = D.decode_drops(raw)
        rows = np.frombuffer(raw.tobytes(), D.DROP_DTYPE)
        conv = go_drop_record
    cols = [batch.src_ip, batch.dst_ip, batch.bytes, batch.meta, batch.ports, batch.dns_id, batch.tcp_id,
            batch.time_ns]
    for i in range(len(rows)):
        assert conv(rows[i]) == tuple(int(c[i]) for c in cols), i


def _normalize(r):
    """A flow carries protocol and ports only for TCP / UDP (ToFlow), and no metric reads
    them for other protocols (side_key, family_matches)."""
    src, dst, nb, meta, ports, dns, tcp_id, t = r
    if meta & 0xFF not in (6, 17):
        meta, ports = meta & ~0xFF, 0
    return (src, dst, nb, meta, ports, dns, tcp_id, t)


@pytest.mark.parametrize("kind", ["packet", "drop"])
def test_adapter_equals_record_constructors(kind):
    """Write(*v1.Event) and the direct path agree: the flow packetparser / dropreason build
    from a sample (oracle.decode_packet / decode_drop, processRecord restated), turned back
    by the adapter, is the record PacketRecord / DropRecord give -- out-of-range directions
    and drop types included (both leave them to verdict 255).  records_linux_test.go runs
    the same comparison in Go with the reference's own utils.ToFlow."""
    import numpy as np
    from oracle import decode as D
    pods = W.make_pods(100, seed=3)
    if kind == "packet":
        raw = W.gen_raw_packets(3000, pods, seed=13, odd_frac=0.3, out_of_range_frac=0.05)
        rows = np.frombuffer(raw.tobytes(), D.PACKET_DTYPE)
        b, sz = raw.tobytes(), D.PACKET_DTYPE.itemsize
        flows = [O.decode_packet(b[i * sz:(i + 1) * sz]) for i in range(len(rows))]
        conv = go_packet_record
    else:
        raw = W.gen_raw_drops(3000, pods, seed=14, out_of_range_frac=0.05)
        rows = np.frombuffer(raw.tobytes(), D.DROP_DTYPE)
        b, sz = raw.tobytes(), D.DROP_DTYPE.itemsize
        flows = [O.decode_drop(b[i * sz:(i + 1) * sz]) for i in range(len(rows))]
        conv = go_drop_record
    n255 = 0
    for i, f in enumerate(flows):
        got = go_flow_to_record(f, None)
        want = conv(rows[i])
        assert got is not None and _normalize(got) == _normalize(want), i
        n255 += (want[3] >> 8 & 0xFF) == 255
    assert n255 > 0
