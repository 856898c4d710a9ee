"""GPU parity of the raw perf-record decode (gpuagg_decode.hip) through the C-ABI.

* decoded columns bit-exact against oracle/decode.py (itself pinned to
  oracle.decode_packet / decode_drop, tests/test_decode_oracle.py), incl. tile tails,
  odd field values and rows that do not fit the meta word;
* decode + aggregate (host-fed and device-resident) against the oracle's per-flow
  replay of the raw records through processRecord -> enrich -> every metric;
* at BASELINE.json's C2 size (100M records): decode(encode(columns)) == columns on the
  device, and raw-path counters == column-path counters.
"""

import numpy as np
import pytest

from oracle import decode as D
from oracle import oracle as O
from oracle import records as R
from retina_amd import workloads as W
from retina_amd import _abi

from .helpers import diff_series, make_engine, oracle_cache

pytestmark = pytest.mark.gpu

SPEC_LOCAL = [{"metric_name": n, "source_labels": ["namespace", "podname"]}
              for n in ["forward_count", "forward_bytes", "drop_count", "drop_bytes", "tcp_flag_gauges"]]
SPEC_REMOTE = [{"metric_name": n, "source_labels": ["ip", "podname", "port"],
                "destination_labels": ["namespace", "workload"]}
               for n in ["forward_count", "forward_bytes", "drop_count", "drop_bytes", "tcp_flag_gauges"]]


def _dev_u8(raw: np.ndarray, dev):
    import torch
    return torch.from_numpy(raw).to(dev)


def _out_cols(n, dev):
    import torch
    return [torch.full((max(n, 1),), 0x5A5A5A5A, dtype=torch.int32, device=dev) for _ in range(6)]


def _np(t, n):
    return t[:n].cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("kind", [_abi.RAW_PACKET, _abi.RAW_DROP], ids=["packet", "drop"])
@pytest.mark.parametrize("n", [1, 511, 512, 513, 100_003])
def test_decode_columns_bitexact(gpu_device, kind, n):
    import torch
    from retina_amd import GpuAgg
    dev = torch.device("cuda", gpu_device)
    pods = W.make_pods(100, seed=1)
    if kind == _abi.RAW_PACKET:
        raw = W.gen_raw_packets(n, pods, seed=n, odd_frac=0.2, out_of_range_frac=0.01)
        want, bad = D.decode_packets(raw)
    else:
        raw = W.gen_raw_drops(n, pods, seed=n, out_of_range_frac=0.01)
        want, bad = D.decode_drops(raw)
    g = make_engine(pods, SPEC_LOCAL, False, gpu_device)
    try:
        d_raw = _dev_u8(raw, dev)
        out = _out_cols(n, dev)
        g.decode_device(kind, d_raw.data_ptr(), n, GpuAgg.device_columns(*out))
        g.sync()
        for name, t, w in zip(("src_ip", "dst_ip", "bytes", "meta", "ports", "dns_id"), out,
                              (want.src_ip, want.dst_ip, want.bytes, want.meta, want.ports, want.dns_id)):
            got = _np(t, n)
            assert np.array_equal(got, w), (name, np.flatnonzero(got != w)[:5])
        assert g.stats()["decode_out_of_range"] == int(bad.sum())
        assert g.stats()["decoded"] == n
    finally:
        g.close()


def _oracle_raw_series(pk, dr, pods, spec, remote):
    m = O.Module(remote_context=remote)
    m.reconcile(R.spec_from_json(spec))
    cache = oracle_cache(pods)
    flows = [O.decode_packet(pk[i * 72:(i + 1) * 72].tobytes()) for i in range(len(pk) // 72)]
    flows += [O.decode_drop(dr[i * 32:(i + 1) * 32].tobytes()) for i in range(len(dr) // 32)]
    for f in flows:
        f = O.enrich(cache, f)
        if f is not None:
            m.process_flow(f)
    return m.series()


@pytest.mark.parametrize("remote", [False, True], ids=["local", "remote"])
@pytest.mark.parametrize("host_fed", [True, False], ids=["host", "device"])
def test_raw_aggregate_vs_oracle(gpu_device, remote, host_fed):
    import torch
    pods = W.make_pods(300, seed=21)
    pk = W.gen_raw_packets(20_000, pods, seed=22, odd_frac=0.1)
    dr = W.gen_raw_drops(6_000, pods, seed=23)
    spec = SPEC_REMOTE if remote else SPEC_LOCAL
    want = _oracle_raw_series(pk, dr, pods, spec, remote)
    g = make_engine(pods, spec, remote, gpu_device)
    try:
        if host_fed:
            g.submit_raw(_abi.RAW_PACKET, pk, chunk=7_000)   # chunks: not multiples of the tile
            g.submit_raw(_abi.RAW_DROP, dr)
        else:
            dev = torch.device("cuda", gpu_device)
            d_pk, d_dr = _dev_u8(pk, dev), _dev_u8(dr, dev)
            g.submit_raw_device(_abi.RAW_PACKET, d_pk.data_ptr(), len(pk) // 72)
            g.submit_raw_device(_abi.RAW_DROP, d_dr.data_ptr(), len(dr) // 32)
            g.sync()
        got = g.snapshot()
    finally:
        g.close()
    assert got == want, diff_series(got, want)


@pytest.mark.parametrize("mode", [_abi.FEED_HOST_DECODE, _abi.FEED_RAW_DMA], ids=["host-decode", "raw-dma"])
@pytest.mark.parametrize("world,threads", [(1, 1), (1, 8), (3, 4)])
@pytest.mark.parametrize("remote", [False, True], ids=["local", "remote"])
def test_raw_feed_vs_oracle(gpu_device, remote, world, threads, mode):
    """The Go plugin's raw path: gpuagg_raw_feed_put over `world` contexts (all on this GPU),
    two pinned stagings per context submitted without waiting for their DMA, samples decoded
    on the feed's threads or on the GPU.  Every context's series equal the oracle over the
    records gpuagg_shard_raw gives it; capacities force many stagings and straddling pieces."""
    import ctypes as C
    from retina_amd import RawFeed
    pods = W.make_pods(300, seed=24)
    pk = W.gen_raw_packets(60_000, pods, seed=25, odd_frac=0.1, out_of_range_frac=0.01)
    dr = W.gen_raw_drops(20_000, pods, seed=26, out_of_range_frac=0.01)
    spec = SPEC_REMOTE if remote else SPEC_LOCAL
    engines = [make_engine(pods, spec, remote, gpu_device) for _ in range(world)]
    feeds = [RawFeed(engines, k, capacity=cap, threads=threads, mode=mode)
             for k, cap in ((_abi.RAW_PACKET, 6_000), (_abi.RAW_DROP, 3_000))]
    try:
        for feed, raw in zip(feeds, (pk, dr)):
            sz = feed.size
            n = len(raw) // sz
            for a in range(0, n, 7_000):
                feed.put(raw[a * sz:min(n, a + 7_000) * sz])
            feed.flush()
        shards = []
        for kind, raw, sz in ((_abi.RAW_PACKET, pk, 72), (_abi.RAW_DROP, dr, 32)):
            sh = np.zeros(len(raw) // sz, np.uint32)
            assert engines[0].lib.gpuagg_shard_raw(kind, raw.ctypes.data_as(C.c_void_p), len(sh), world,
                                                   sh.ctypes.data_as(_abi.u32p)) == 0
            shards.append(sh)
        assert feeds[0].submitted() == [int((shards[0] == d).sum()) for d in range(world)]
        _, bad_p = D.decode_packets(pk)
        _, bad_d = D.decode_drops(dr)
        for d, g in enumerate(engines):
            mp, md = shards[0] == d, shards[1] == d
            # out-of-range rows are counted and consumed by no metric (the oracle would label them)
            want = _oracle_raw_series(pk.reshape(-1, 72)[mp & ~bad_p].reshape(-1),
                                      dr.reshape(-1, 32)[md & ~bad_d].reshape(-1), pods, spec, remote)
            got = g.snapshot()
            assert got == want, diff_series(got, want)
            assert g.stats()["decode_out_of_range"] == int(bad_p[mp].sum() + bad_d[md].sum())
    finally:
        for f in feeds:
            f.close()
        for g in engines:
            g.close()


def test_unencodable_rows_are_not_aggregated(gpu_device):
    """traffic_direction > 3 / drop_type > 7: counted, consumed by no metric."""
    pods = W.make_pods(100, seed=31)
    pk = W.gen_raw_packets(8_000, pods, seed=32, out_of_range_frac=0.05)
    dr = W.gen_raw_drops(4_000, pods, seed=33, out_of_range_frac=0.05)
    bp, badp = D.decode_packets(pk)
    bd, badd = D.decode_drops(dr)
    m = O.Module(remote_context=False)
    m.reconcile(R.spec_from_json(SPEC_LOCAL))
    cache = oracle_cache(pods)
    R.replay(R.Batch(bp.src_ip[~badp], bp.dst_ip[~badp], bp.bytes[~badp], bp.meta[~badp], bp.ports[~badp]), cache, m)
    R.replay(R.Batch(bd.src_ip[~badd], bd.dst_ip[~badd], bd.bytes[~badd], bd.meta[~badd], bd.ports[~badd]), cache, m)
    g = make_engine(pods, SPEC_LOCAL, False, gpu_device)
    try:
        g.submit_raw(_abi.RAW_PACKET, pk)
        g.submit_raw(_abi.RAW_DROP, dr)
        g.sync()
        assert g.stats()["decode_out_of_range"] == int(badp.sum() + badd.sum())
        got = g.snapshot()
    finally:
        g.close()
    want = m.series()
    assert got == want, diff_series(got, want)


def test_bad_arguments(gpu_device):
    import torch
    from retina_amd import GpuAgg, GpuAggError
    pods = W.make_pods(10, seed=1)
    g = make_engine(pods, SPEC_LOCAL, False, gpu_device)
    try:
        dev = torch.device("cuda", gpu_device)
        raw = torch.zeros(72 * 4 + 16, dtype=torch.uint8, device=dev)
        out = GpuAgg.device_columns(*_out_cols(4, dev))
        with pytest.raises(GpuAggError):
            g.decode_device(3, raw.data_ptr(), 4, out)                 # unknown kind
        with pytest.raises(GpuAggError):
            g.decode_device(_abi.RAW_PACKET, raw.data_ptr() + 4, 4, out)  # misaligned
        with pytest.raises(ValueError):
            g.submit_raw(_abi.RAW_DROP, np.zeros(33, np.uint8))         # ragged buffer
        g.decode_device(_abi.RAW_PACKET, raw.data_ptr(), 0, out)         # empty: no-op
        g.submit_raw(_abi.RAW_DROP, np.zeros(0, np.uint8))
        assert g.snapshot() == {}
    finally:
        g.close()


def test_full_size_raw_roundtrip(gpu_device):
    """C2 size: 100M packetparser records encoded on the device from the C2 columns
    (verdict forced FORWARDED); decode(encode(cols)) == cols and raw-path counters ==
    column-path counters, bit for bit."""
    import torch
    from retina_amd import GpuAgg
    dev = torch.device("cuda", gpu_device)
    pods = W.make_pods(10_000, seed=2)
    n, chunk = 100_000_000, 10_000_000
    cols = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(5)]
    for k in range(n // chunk):
        r = W.gen_records(chunk, pods, seed=5000 + k, udp_frac=0.1, other_proto_frac=0.02)
        proto, flags = r.meta & 0xFF, (r.meta >> 21) & 0x3F
        tdir, rep = (r.meta >> 16) & 3, (r.meta >> 27) & 1
        meta = W.pack_meta(proto, 1, tdir, 0, np.where(proto == 6, flags, 0), rep, 0, obs=2)  # encoder: obs 2
        for t, a in zip(cols, (r.src_ip, r.dst_ip, r.bytes, meta, r.ports)):
            t[k * chunk:(k + 1) * chunk].copy_(torch.from_numpy(np.ascontiguousarray(a).view(np.int32)))
    raw = W.raw_packets_torch(*cols)
    spec = [{"metric_name": x, "source_labels": ["namespace", "podname"]}
            for x in ["forward_count", "forward_bytes", "tcp_flag_gauges"]]
    g1 = make_engine(pods, spec, False, gpu_device)
    g2 = make_engine(pods, spec, False, gpu_device)
    try:
        out = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(6)]
        g1.decode_device(_abi.RAW_PACKET, raw.data_ptr(), n, GpuAgg.device_columns(*out))
        g1.sync()
        for a, b in zip(out[:5], cols):
            assert torch.equal(a, b)
        assert bool((out[5] == -1).all())
        del out
        g1.submit_raw_device(_abi.RAW_PACKET, raw.data_ptr(), n)
        got = g1.snapshot()
        g2.submit_device(GpuAgg.device_columns(*cols), n)
        want = g2.snapshot()
    finally:
        g1.close()
        g2.close()
    assert got == want, diff_series(got, want)
