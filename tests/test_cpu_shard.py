"""The library's host sharding (gpuagg_shard_raw / gpuagg_shard_columns, used by the Go
plugin to spread raw perf records and decoded records over the node's devices) equals
retina_amd/dist.py shard_of on the decoded columns: one function on every side."""

import ctypes as C

import numpy as np
import pytest

from oracle import decode as D
from retina_amd import dist
from retina_amd import workloads as W


@pytest.fixture(scope="module")
def lib():
    from retina_amd import _abi, build
    build.build()
    return _abi.load()


def _u32p(a):
    from retina_amd import _abi
    return a.ctypes.data_as(_abi.u32p)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_raw_and_columns_match_dist(lib, world):
    from retina_amd import _abi
    pods = W.make_pods(500, seed=3)
    for kind, raw, dec in ((_abi.RAW_PACKET, W.gen_raw_packets(20_000, pods, seed=4, odd_frac=0.05), D.decode_packets),
                           (_abi.RAW_DROP, W.gen_raw_drops(20_000, pods, seed=5), D.decode_drops)):
        b, _ = dec(raw)
        n = len(b.src_ip)
        want = dist.shard_of(b.src_ip, b.dst_ip, b.ports, b.meta, world)
        got = np.zeros(n, np.uint32)
        assert lib.gpuagg_shard_raw(kind, raw.ctypes.data_as(C.c_void_p), n, world, _u32p(got)) == 0
        assert np.array_equal(got, want), kind
        cols = [np.ascontiguousarray(x, np.uint32) for x in (b.src_ip, b.dst_ip, b.ports, b.meta)]
        got2 = np.zeros(n, np.uint32)
        assert lib.gpuagg_shard_columns(*[_u32p(x) for x in cols], n, world, _u32p(got2)) == 0
        assert np.array_equal(got2, want)
        assert len(set(got.tolist())) == world  # every shard gets records


def test_mirrored_tuple_same_shard(lib):
    """A request and its mirrored reply land on one shard (the latency join needs both)."""
    rng = np.random.default_rng(9)
    n = 5000
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    sp = rng.integers(0, 65536, n, dtype=np.uint32)
    dp = rng.integers(0, 65536, n, dtype=np.uint32)
    meta = np.full(n, 6, np.uint32)
    a, b = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
    fwd = [src, dst, (sp | (dp << 16)).astype(np.uint32), meta]
    rev = [dst, src, (dp | (sp << 16)).astype(np.uint32), meta]
    assert lib.gpuagg_shard_columns(*[_u32p(x) for x in fwd], n, 8, _u32p(a)) == 0
    assert lib.gpuagg_shard_columns(*[_u32p(x) for x in rev], n, 8, _u32p(b)) == 0
    assert np.array_equal(a, b)


def test_bad_arguments(lib):
    from retina_amd import _abi
    out = np.zeros(1, np.uint32)
    raw = np.zeros(72, np.uint8)
    assert lib.gpuagg_shard_raw(99, raw.ctypes.data_as(C.c_void_p), 1, 2, _u32p(out)) == _abi.EINVAL
    assert lib.gpuagg_shard_raw(_abi.RAW_PACKET, raw.ctypes.data_as(C.c_void_p), 1, 0, _u32p(out)) == _abi.EINVAL


@pytest.mark.parametrize("world,cap,threads,mode", [(1, 5_000, 1, 0), (1, 5_000, 8, 0), (1, 5_000, 3, 1),
                                                    (3, 4_096, 4, 0), (3, 4_096, 1, 1), (8, 1_000, 8, 0),
                                                    (8, 1_000, 5, 1)])
def test_raw_feed_scatter(lib, world, cap, threads, mode):
    """gpuagg_raw_feed_* (the Go plugin's node-wide raw path) on CPU-backend contexts:
    every context receives exactly the records gpuagg_shard_raw assigns it, its series
    equal the oracle over that shard, and the merged state equals one context fed
    everything.  Capacities smaller than the input force submits in the middle of a put
    (and pieces that straddle the two stagings); host-decoded (mode 0) and raw-copied
    (mode 1, decoded by the context) samples, one and several feed threads."""
    from retina_amd import RawFeed, _abi
    from .helpers import diff_series, make_engine, oracle_series
    pods = W.make_pods(300, seed=21)
    sp = [{"metric_name": m, "source_labels": ["namespace", "podname"]}
          for m in ("forward_count", "forward_bytes", "drop_count", "drop_bytes")]
    for kind, raw, dec in ((_abi.RAW_PACKET, W.gen_raw_packets(12_000, pods, seed=22), D.decode_packets),
                           (_abi.RAW_DROP, W.gen_raw_drops(9_000, pods, seed=23), D.decode_drops)):
        b, _ = dec(raw)
        n = len(b.src_ip)
        shard = np.zeros(n, np.uint32)
        assert lib.gpuagg_shard_raw(kind, raw.ctypes.data_as(C.c_void_p), n, world, _u32p(shard)) == 0
        engines = [make_engine(pods, sp, False, flags=_abi.FLAG_CPU_BACKEND) for _ in range(world)]
        feed = RawFeed(engines, kind, capacity=cap, threads=threads, mode=mode)
        try:
            step = 2_500  # several puts, unaligned with the capacity
            for a in range(0, n, step):
                feed.put(raw[a * feed.size:min(n, a + step) * feed.size])
            feed.flush()
            assert feed.submitted() == [int((shard == d).sum()) for d in range(world)]
            for d, g in enumerate(engines):
                m = shard == d
                part = W.Records(b.src_ip[m], b.dst_ip[m], b.bytes[m], b.meta[m], b.ports[m], b.dns_id[m])
                want = oracle_series(part, pods, sp, False)
                got = g.snapshot()
                assert got == want, diff_series(got, want)
            st = [g.stats() for g in engines]
            assert sum(x["decoded"] for x in st) == n
            assert sum(x["decode_out_of_range"] for x in st) == 0
        finally:
            feed.close()
            for g in engines:
                g.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_raw_feed_out_of_range_rows_counted(lib, mode):
    """Rows whose traffic direction does not fit the meta word are counted in
    gpuagg_stats.decode_out_of_range whichever side decodes them, and feed no metric."""
    from retina_amd import RawFeed, _abi
    from .helpers import diff_series, make_engine, oracle_series
    pods = W.make_pods(100, seed=41)
    sp = [{"metric_name": "forward_count", "source_labels": ["namespace", "podname"]}]
    raw = W.gen_raw_packets(6_000, pods, seed=42, out_of_range_frac=0.05)
    b, bad = D.decode_packets(raw)
    g = make_engine(pods, sp, False, flags=_abi.FLAG_CPU_BACKEND)
    feed = RawFeed([g], _abi.RAW_PACKET, capacity=2_000, threads=4, mode=mode)
    try:
        feed.put(raw)
        feed.flush()
        g.sync()
        assert g.stats()["decode_out_of_range"] == int(bad.sum()) > 0
        part = W.Records(b.src_ip, b.dst_ip, b.bytes, b.meta, b.ports, b.dns_id)
        want = oracle_series(part, pods, sp, False)
        got = g.snapshot()
        assert got == want, diff_series(got, want)
    finally:
        feed.close()
        g.close()


def test_raw_feed_after_context_destroy(lib):
    """gpuagg_destroy detaches the feeds over the context: later puts and flushes return
    GPUAGG_ESTATE, and the feed's own destroy is still safe (no use after free)."""
    from retina_amd import GpuAggError, RawFeed, _abi
    from .helpers import make_engine
    pods = W.make_pods(50, seed=43)
    sp = [{"metric_name": "forward_count", "source_labels": ["namespace", "podname"]}]
    raw = W.gen_raw_packets(1_000, pods, seed=44)
    engines = [make_engine(pods, sp, False, flags=_abi.FLAG_CPU_BACKEND) for _ in range(2)]
    feed = RawFeed(engines, _abi.RAW_PACKET, capacity=4_096)
    feed.put(raw)
    engines[1].close()
    with pytest.raises(GpuAggError) as e:
        feed.put(raw)
    assert e.value.code == _abi.ESTATE
    with pytest.raises(GpuAggError):
        feed.flush()
    feed.close()
    engines[0].close()


def test_raw_feed_configure_needs_an_empty_feed(lib):
    from retina_amd import GpuAggError, RawFeed, _abi
    from .helpers import make_engine
    pods = W.make_pods(50, seed=45)
    sp = [{"metric_name": "forward_count", "source_labels": ["namespace", "podname"]}]
    g = make_engine(pods, sp, False, flags=_abi.FLAG_CPU_BACKEND)
    feed = RawFeed([g], _abi.RAW_PACKET, capacity=4_096)
    try:
        feed.put(W.gen_raw_packets(100, pods, seed=46))
        with pytest.raises(GpuAggError) as e:
            feed.configure(4, _abi.FEED_RAW_DMA)
        assert e.value.code == _abi.ESTATE
        feed.flush()
        feed.configure(4, _abi.FEED_RAW_DMA)
        assert lib.gpuagg_raw_feed_configure(feed.h, 0, 7) == _abi.EINVAL
    finally:
        feed.close()
        g.close()


def test_raw_feed_rejects_bad_args(lib):
    from retina_amd import _abi
    h = C.c_void_p()
    arr = (C.c_void_p * 1)(None)
    assert lib.gpuagg_raw_feed_create(arr, 1, _abi.RAW_PACKET, 16, C.byref(h)) == _abi.EINVAL
    assert lib.gpuagg_raw_feed_put(None, None, 0) == _abi.EINVAL
    assert lib.gpuagg_raw_feed_flush(None) == _abi.EINVAL


@pytest.mark.parametrize("world,cap", [(1, 7_000), (3, 2_048)])
def test_record_feed_scatter(lib, world, cap):
    """GPUAGG_RECORD feed (the Go plugin's WriteBatch slices of Record): AoS records sharded
    by gpuagg_shard_columns' function and transposed into each context's pinned SoA batch;
    every context's series equal the oracle over its shard."""
    from retina_amd import RawFeed, _abi
    from retina_amd.engine import records_aos
    from .helpers import diff_series, make_engine, oracle_series
    pods = W.make_pods(300, seed=31)
    sp = [{"metric_name": m, "source_labels": ["namespace", "podname"]}
          for m in ("forward_count", "forward_bytes", "drop_count", "drop_bytes")]
    recs = W.gen_records(20_000, pods, seed=32, drop_frac=0.2, udp_frac=0.1)
    aos = records_aos(recs)
    shard = dist.shard_of(recs.src_ip, recs.dst_ip, recs.ports, recs.meta, world)
    engines = [make_engine(pods, sp, False, flags=_abi.FLAG_CPU_BACKEND) for _ in range(world)]
    feed = RawFeed(engines, _abi.RECORD, capacity=cap)
    try:
        for a in range(0, len(aos), 3_000):
            feed.put(aos[a:a + 3_000])
        feed.flush()
        assert feed.submitted() == [int((shard == d).sum()) for d in range(world)]
        for d, g in enumerate(engines):
            m = shard == d
            part = W.Records(recs.src_ip[m], recs.dst_ip[m], recs.bytes[m], recs.meta[m], recs.ports[m],
                             recs.dns_id[m])
            want = oracle_series(part, pods, sp, False)
            got = g.snapshot()
            assert got == want, diff_series(got, want)
    finally:
        feed.close()
        for g in engines:
            g.close()


def test_feeds_share_one_thread_pool(lib):
    """The plugin's packet, drop and record feeds over the same contexts share one pool of
    host threads (three pools of up to 16 spinning threads each before), and the
    shared pool still scatters every feed's records exactly."""
    import os
    from retina_amd import RawFeed, _abi
    from .helpers import make_engine
    pods = W.make_pods(80, seed=47)
    sp = [{"metric_name": "forward_count", "source_labels": ["namespace", "podname"]}]
    engines = [make_engine(pods, sp, False, flags=_abi.FLAG_CPU_BACKEND) for _ in range(2)]
    threads = lambda: len(os.listdir("/proc/self/task"))  # noqa: E731
    before = threads()
    feeds = [RawFeed(engines, kind, capacity=2_048, threads=6)
             for kind in (_abi.RAW_PACKET, _abi.RAW_DROP, _abi.RECORD)]
    # one pool of 6: the caller's thread + 5 workers (three pools would add 15).  Under the
    # sanitizer preload (test_sanitize.py) the runtime may start one thread of its own at
    # the first thread creation, here or earlier
    extra = threads() - before - 5
    assert 0 <= extra <= (1 if "san" in os.environ.get("LD_PRELOAD", "") else 0), extra
    raw = W.gen_raw_packets(5_000, pods, seed=48)
    feeds[0].put(raw)
    feeds[0].flush()
    assert sum(feeds[0].submitted()) == 5_000
    for f in feeds:
        f.close()
    assert threads() - before == extra  # the last feed joined the pool's workers
    for e in engines:
        e.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_raw_feed_dry_run_counts_only(lib, mode):
    """GPUAGG_FEED_DRY_RUN (the bench's host-only ceiling): every record is sharded and
    counted as submitted, nothing is aggregated; a later configure without it feeds again."""
    from retina_amd import RawFeed, _abi
    from .helpers import make_engine
    pods = W.make_pods(60, seed=49)
    sp = [{"metric_name": "forward_count", "source_labels": ["namespace", "podname"]}]
    engines = [make_engine(pods, sp, False, flags=_abi.FLAG_CPU_BACKEND) for _ in range(3)]
    raw = W.gen_raw_packets(9_000, pods, seed=50)
    feed = RawFeed(engines, _abi.RAW_PACKET, capacity=1_024, threads=3, mode=mode | _abi.FEED_DRY_RUN)
    feed.put(raw)
    feed.flush()
    assert sum(feed.submitted()) == 9_000
    assert all(e.snapshot() == {} for e in engines)
    feed.configure(3, mode)
    feed.put(raw)
    feed.flush()
    assert sum(feed.submitted()) == 18_000
    assert any(e.snapshot() for e in engines)
    feed.close()
    for e in engines:
        e.close()
