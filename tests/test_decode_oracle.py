"""Raw perf-record decode: the numpy restatement (oracle/decode.py) pinned to the
per-record restatements oracle.decode_packet / oracle.decode_drop and to the
reference's own test inputs (CPU only).

Known answers from the reference's tests:
* dropreason_linux_test.go:211-215 feeds a raw sample whose byte i is i (32 bytes)
  through processRecord and expects one enricher.Write; decoded here field by field.
* packetparser_linux_test.go:314-321 builds packetparserPacket{SrcIp 83886272
  (192.0.0.5), DstIp 16777226 (10.0.0.1), Proto 6, ObservationPoint 1, SrcPort 80,
  DstPort 443}; its binary layout is decoded here (the test itself JSON-encodes it).
"""

import numpy as np
import pytest

from oracle import decode as D
from oracle import oracle as O
from oracle import records as R
from retina_amd import workloads as W

from .helpers import oracle_cache


def _flow_fields(f: O.Flow):
    l4 = None if f.l4 is None else (f.l4.proto, f.l4.source_port, f.l4.destination_port, f.l4.flags)
    ext = f.extensions
    return (f.ip.source, f.ip.destination, l4, f.verdict, f.traffic_direction, ext.bytes,
            ext.drop_reason, f.trace_observation_point if f.trace_observation_point in
            (O.OBS_TO_NETWORK, O.OBS_FROM_NETWORK) else None, ext.tcp_id, f.time_ns)


def _check_rows(batch: R.Batch, bad: np.ndarray, flows):
    for i, f in enumerate(flows):
        if bad[i]:
            assert (int(batch.meta[i]) >> 8) & 0xFF == 255
            continue
        g = R.flow_from_record(int(batch.src_ip[i]), int(batch.dst_ip[i]), int(batch.bytes[i]),
                               int(batch.meta[i]), int(batch.ports[i]), 0, {}, int(batch.tcp_id[i]),
                               int(batch.time_ns[i]))
        assert _flow_fields(g) == _flow_fields(f), i
        if f.is_reply is not None:
            assert bool(f.is_reply) == bool((int(batch.meta[i]) >> 27) & 1), i


def test_packet_decode_matches_per_record_oracle():
    pods = W.make_pods(200, seed=3)
    raw = W.gen_raw_packets(4000, pods, seed=5, odd_frac=0.3, out_of_range_frac=0.03)
    batch, bad = D.decode_packets(raw)
    flows = [O.decode_packet(raw[i * 72:(i + 1) * 72].tobytes()) for i in range(len(batch))]
    assert 0 < bad.sum() < len(batch)
    _check_rows(batch, bad, flows)


def test_drop_decode_matches_per_record_oracle():
    pods = W.make_pods(200, seed=3)
    raw = W.gen_raw_drops(4000, pods, seed=6, out_of_range_frac=0.03)
    batch, bad = D.decode_drops(raw)
    flows = [O.decode_drop(raw[i * 32:(i + 1) * 32].tobytes()) for i in range(len(batch))]
    assert 0 < bad.sum() < len(batch)
    _check_rows(batch, bad, flows)


def test_dropreason_reference_raw_sample():
    """dropreason_linux_test.go:211-215: rawSample[i] = byte(i)."""
    raw = np.arange(32, dtype=np.uint8)
    f = O.decode_drop(raw.tobytes())
    assert (f.ip.source, f.ip.destination) == ("0.1.2.3", "4.5.6.7")
    assert f.l4 is None                       # proto 0x16 = 22: neither TCP nor UDP
    assert f.verdict == O.VERDICT_DROPPED and f.traffic_direction == O.TD_INGRESS
    assert f.extensions.bytes == 0x0F0E0D0C and f.extensions.drop_reason == 0x1514
    batch, bad = D.decode_drops(raw)
    assert bool(bad[0])                       # drop_type 5396 does not fit the meta word
    assert int(batch.src_ip[0]) == O.ip2int("0.1.2.3") and int(batch.bytes[0]) == 0x0F0E0D0C
    assert int(batch.ports[0]) == (0x0809 | (0x0A0B << 16))   # HostToNetShort(0x0908), (0x0B0A)


def test_packetparser_reference_event():
    """packetparser_linux_test.go:314-321 field values in the binary layout."""
    r = np.zeros(1, W.RAW_PACKET_DTYPE)
    r["src_ip"], r["dst_ip"], r["proto"], r["obs"] = 83886272, 16777226, 6, 1
    r["src_port"], r["dst_port"] = 80, 443
    raw = r.view(np.uint8)
    f = O.decode_packet(raw.tobytes())
    assert (f.ip.source, f.ip.destination) == ("192.0.0.5", "10.0.0.1")
    assert f.l4.proto == "TCP" and (f.l4.source_port, f.l4.destination_port) == (20480, 47873)
    assert f.trace_observation_point == O.OBS_TO_ENDPOINT and f.verdict == O.VERDICT_FORWARDED
    batch, bad = D.decode_packets(raw)
    assert not bad[0]
    _check_rows(batch, bad, [f])


@pytest.mark.parametrize("remote", [False, True])
def test_series_raw_replay_equals_column_replay(remote):
    """Whole metrics pipeline: flows from the per-record decoders vs the decoded batch."""
    pods = W.make_pods(150, seed=9)
    pk = W.gen_raw_packets(2500, pods, seed=10, odd_frac=0.2)
    dr = W.gen_raw_drops(1500, pods, seed=11)
    spec = [{"metric_name": n, "source_labels": ["namespace", "podname", "port"],
             "destination_labels": ["ip", "workload"] if remote else None}
            for n in ["forward_count", "forward_bytes", "drop_count", "drop_bytes", "tcp_flag_gauges"]]
    cache = oracle_cache(pods)

    m1 = O.Module(remote_context=remote)
    m1.reconcile(R.spec_from_json(spec))
    flows = [O.decode_packet(pk[i * 72:(i + 1) * 72].tobytes()) for i in range(len(pk) // 72)]
    flows += [O.decode_drop(dr[i * 32:(i + 1) * 32].tobytes()) for i in range(len(dr) // 32)]
    for f in flows:
        f = O.enrich(cache, f)
        if f is not None:
            m1.process_flow(f)

    m2 = O.Module(remote_context=remote)
    m2.reconcile(R.spec_from_json(spec))
    for raw, dec in ((pk, D.decode_packets), (dr, D.decode_drops)):
        b, bad = dec(raw)
        assert not bad.any()
        R.replay(b, cache, m2)
    assert m1.series() == m2.series()
