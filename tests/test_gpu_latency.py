"""Node-apiserver latency on the GPU (gpuagg_latency.hip) against the restated TTL join
(oracle/latency.py, pinned to latency_test.go's cases in tests/test_latency_oracle.py):
device columns in one batch and in several (requests carried across batches), host-fed
batches, the raw packetparser decode path, and the text exposition."""

import numpy as np
import pytest

from oracle import latency as L
from oracle import oracle as O
from retina_amd import workloads as W

from .helpers import make_engine
from .latency_helpers import as_state, oracle_latency

pytestmark = pytest.mark.gpu

API = [W.ip_le(10, 255, 0, 1), W.ip_le(10, 255, 0, 2)]
SPEC = [{"metric_name": "node_apiserver_latency"}, {"metric_name": "node_apiserver_handshake_latency"},
        {"metric_name": "node_apiserver_no_response"},
        {"metric_name": "forward_count", "source_labels": ["namespace", "podname"]}]


def _dev(recs, device):
    import torch
    dev = torch.device("cuda", device)

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    return [t(recs.src_ip), t(recs.dst_ip), t(recs.bytes), t(recs.meta), t(recs.ports), t(recs.dns_id),
            t(recs.tcp_id), torch.from_numpy(np.ascontiguousarray(recs.time_ns).view(np.int64)).to(dev)]


def _engine(pods, device):
    g = make_engine(pods, SPEC, False, device)
    g.set_apiserver_ips(API)
    return g


def _state(g):
    st = g.latency_state()
    return {k: st[k] for k in ("latency_buckets", "latency_count", "latency_sum", "handshake_buckets",
                               "handshake_count", "handshake_sum", "no_response", "pending")}


@pytest.mark.parametrize("chunks", [1, 3, 17])
def test_device_batches_match_oracle(gpu_device, chunks):
    from retina_amd import GpuAgg
    pods = W.make_pods(100, seed=11)
    recs = W.gen_latency_records(400, pods, API, seed=12, background=3000)
    want = as_state(oracle_latency(recs, API))
    g = _engine(pods, gpu_device)
    try:
        ts = _dev(recs, gpu_device)
        n = len(recs.src_ip)
        bounds = np.linspace(0, n, chunks + 1).astype(int)
        for a, b in zip(bounds[:-1], bounds[1:]):
            g.submit_device(GpuAgg.device_columns(*[x[a:] for x in ts]), int(b - a))
        got = _state(g)
    finally:
        g.close()
    assert got == want
    assert want["latency_count"] > 0 and want["no_response"] > 0 and want["pending"] > 0


def test_host_fed_and_text(gpu_device):
    pods = W.make_pods(100, seed=21)
    recs = W.gen_latency_records(200, pods, API, seed=22, background=1000)
    m = oracle_latency(recs, API)
    g = _engine(pods, gpu_device)
    try:
        n = len(recs.src_ip)
        hb = g.alloc_batch(n)
        hb.fill(recs)
        g.submit(hb, n)
        g.sync()
        got = _state(g)
        text = g.snapshot_text()
    finally:
        g.close()
    assert got == as_state(m)
    want_text = L.render(m)
    for fam in want_text.split("# HELP ")[1:]:  # each latency family block appears verbatim
        assert "# HELP " + fam in text
    assert "networkobservability_adv_forward_count" in text


@pytest.mark.parametrize("path", ["device", "feed-host-decode", "feed-raw-dma"])
def test_raw_packet_decode_path(gpu_device, path):
    """72-byte packetparser records: TcpId from TSval / TSecr by observation point, the
    time from t_nsec + the monotonic offset -- decoded on the GPU from device memory, or
    handed to a raw feed (decoded on its host threads, or copied and decoded on the GPU)
    in pieces across several 256-record stagings (requests carried between batches)."""
    from retina_amd import RawFeed, _abi
    import torch
    pods = W.make_pods(100, seed=31)
    recs = W.gen_latency_records(150, pods, API, seed=32, background=500)
    off = 123_456_789
    n = len(recs.src_ip)
    raw = np.zeros((n, 72), np.uint8)
    obs = (recs.meta >> 30) & 3
    flags = (recs.meta >> 21) & 0x3F
    tsval = np.where(obs == 3, recs.tcp_id, 7).astype(np.uint32)
    tsecr = np.where(obs == 2, recs.tcp_id, 9).astype(np.uint32)
    t_nsec = (recs.time_ns - np.uint64(off)).astype(np.uint64)
    sport, dport = recs.ports & 0xFFFF, recs.ports >> 16
    swap = lambda x: (((x & 0xFF) << 8) | (x >> 8)).astype(np.uint16)  # noqa: E731  (LE bytes of a net-order short)
    for i in range(n):
        O.PACKET_STRUCT.pack_into(raw[i], 0, int(t_nsec[i]), 100, int(recs.src_ip[i]), int(recs.dst_ip[i]),
                                  int(swap(sport[i])), int(swap(dport[i])), 0, 0, int(tsval[i]), int(tsecr[i]),
                                  int(obs[i]), 2 if obs[i] == 3 else 1, 6, int(flags[i]), False, 0, 0, 0, 0)
    want = as_state(oracle_latency(recs, API))
    g = _engine(pods, gpu_device)
    try:
        g.set_time_offset(off)
        if path == "device":
            d = torch.from_numpy(raw.reshape(-1)).to(torch.device("cuda", gpu_device))
            g.submit_raw_device(_abi.RAW_PACKET, d.data_ptr(), n)
        else:
            mode = _abi.FEED_HOST_DECODE if path == "feed-host-decode" else _abi.FEED_RAW_DMA
            feed = RawFeed([g], _abi.RAW_PACKET, capacity=256, threads=4, mode=mode)
            try:
                flat = raw.reshape(-1)
                for a in range(0, n, 100):
                    feed.put(flat[a * 72:min(n, a + 100) * 72])
                feed.flush()
            finally:
                feed.close()
        got = _state(g)
    finally:
        g.close()
    assert got == want


def test_sharded_contexts_merge(gpu_device):
    """Two contexts fed the direction-free shards (dist.shard_records) and merged equal one
    context: the histograms exactly; no_response + pending as a sum (each shard's clock
    is its own records' running max, so an entry expiring in the last milliseconds of the
    stream may still be pending on one side)."""
    from retina_amd import GpuAgg
    from retina_amd import dist as D
    pods = W.make_pods(100, seed=41)
    recs = W.gen_latency_records(300, pods, API, seed=42, background=2000)
    want = as_state(oracle_latency(recs, API))
    parts = [_engine(pods, gpu_device) for _ in range(2)]
    try:
        for r, g in enumerate(parts):
            sh = D.shard_records(recs, 2, r)
            g.submit_device(GpuAgg.device_columns(*_dev(sh, gpu_device)), len(sh.src_ip))
        parts[0].merge_from(parts[1:])
        got = _state(parts[0])
        rest = _state(parts[1])
    finally:
        for g in parts:
            g.close()
    for k in ("latency_buckets", "latency_count", "latency_sum", "handshake_buckets", "handshake_count",
              "handshake_sum"):
        assert got[k] == want[k], k
    assert got["no_response"] + got["pending"] + rest["pending"] == want["no_response"] + want["pending"]
    assert rest["latency_count"] == 0 and rest["no_response"] == 0  # reset after the merge


def test_apiserver_and_ipcache_before_endpoints(gpu_device):
    """The Go agent's order: the apiserver IPs and the Hubble ipcache are set before the
    IP cache commits its first endpoints, and the endpoint set then grows (the LDS IP
    images are rebuilt larger).  Latency batches and a Hubble decode after the growth
    must still use live buffers and match the oracle."""
    import torch
    from retina_amd import GpuAgg
    small = W.make_pods(50, seed=71)
    big = W.make_pods(3000, seed=71)
    recs = W.gen_latency_records(300, big, API, seed=72, background=2000)
    want = as_state(oracle_latency(recs, API))
    g = GpuAgg(device=gpu_device, max_slots=len(big.endpoints) + 64, max_ips=len(big.ips) + 64,
               sparse_capacity_log2=20, cms_depth=2, cms_width_log2=12, hll_precision=10)
    try:
        g.reconcile(SPEC)
        g.set_apiserver_ips(API)
        ips = big.ips.tolist()
        g.ipcache_set(ips, [1000 + i for i in range(len(ips))], list(range(len(ips))))
        g.load_endpoints(small.endpoints, version=1)  # first commit: the images are built
        g.load_endpoints(big.endpoints, version=2)    # growth: the images are reallocated
        ts = _dev(recs, gpu_device)
        n = len(recs.src_ip)
        half = n // 2
        g.submit_device(GpuAgg.device_columns(*ts), half)
        g.submit_device(GpuAgg.device_columns(*[x[half:] for x in ts]), n - half)
        got = _state(g)
        out = [torch.empty(n, dtype=torch.int32, device=ts[0].device) for _ in range(6)]
        g.hubble_decode_device(GpuAgg.device_columns(*ts), n, out)
        g.sync()
        sid = out[0].cpu().numpy().view(np.uint32)
    finally:
        g.close()
    assert got == want
    pos = {ip: i for i, ip in enumerate(ips)}
    exp = np.array([1000 + pos[int(s)] if int(s) in pos else 2 for s in recs.src_ip], np.uint32)
    assert np.array_equal(sid, exp)


@pytest.mark.parametrize("limit,chunks", [(300, 1), (300, 5), (100_000, 1), (100_000, 3)],
                         ids=["small-1", "small-5", "LIMIT-1", "LIMIT-3"])
def test_capacity_and_touch_match_oracle(gpu_device, limit, chunks):
    """The ttlcache capacity (latency.go LIMIT = 100000, and a small latency_limit) and
    its touch on a Get hit: a burst keeps more requests live than the limit, so the
    batches where the capacity binds run the sequential pass (least recently touched
    evicted, uncounted) and the others the parallel walk; exact against the oracle across
    batches (carried entries keep their LRU order)."""
    from retina_amd import GpuAgg
    from .latency_helpers import as_state
    n_req = 1_200 if limit < 1000 else 130_000
    recs = W.gen_latency_burst(n_req, API, seed=limit + chunks, spacing_ns=100_000 if limit < 1000 else 1_000,
                               background=2_000)
    m = oracle_latency(recs, API, limit=limit)
    want = as_state(m, capacity=True)
    assert want["capacity_evictions"] > 0 and want["peak_live"] == limit
    pods = W.make_pods(50, seed=3)
    g = make_engine(pods, SPEC, False, gpu_device, latency_limit=0 if limit == 100_000 else limit)
    try:
        g.set_apiserver_ips(API)
        ts = _dev(recs, gpu_device)
        n = len(recs.src_ip)
        bounds = np.linspace(0, n, chunks + 1).astype(int)
        for a, b in zip(bounds[:-1], bounds[1:]):
            g.submit_device(GpuAgg.device_columns(*[x[a:] for x in ts]), int(b - a))
        st = g.latency_state()
    finally:
        g.close()
    assert {k: st[k] for k in want} == want
    assert st["limit"] == limit and st["capacity_batches"] >= 1
    assert want["latency_buckets"][10] > 0  # replies kept alive by the touch


def test_touch_without_capacity(gpu_device):
    """Below the capacity (the parallel walk): repeated requests touch their entry, so a
    reply 650 ms after the first packet is observed, as the oracle's ttlcache does."""
    from retina_amd import GpuAgg
    recs = W.gen_latency_burst(3_000, API, seed=5, spacing_ns=50_000, touch_frac=0.2, background=1_000)
    want = as_state(oracle_latency(recs, API), capacity=True)
    assert want["capacity_evictions"] == 0 and want["latency_buckets"][10] > 0
    pods = W.make_pods(50, seed=3)
    g = _engine(pods, gpu_device)
    try:
        g.submit_device(GpuAgg.device_columns(*_dev(recs, gpu_device)), len(recs.src_ip))
        st = g.latency_state()
    finally:
        g.close()
    assert {k: st[k] for k in want} == want
    assert st["capacity_batches"] == 0


@pytest.mark.parametrize("cpu", [False, True], ids=["gpu", "cpu-backend"])
def test_merge_capacity_counters(gpu_device, cpu):
    """gpuagg_merge combines the capacity diagnostics the way a single context would report
    them: capacity_evictions and capacity_batches summed, peak_live the max over
    the contexts; the merged-from context restarts them with its histograms."""
    from retina_amd import _abi
    from retina_amd import dist as D
    from retina_amd import GpuAgg
    pods = W.make_pods(100, seed=51)
    recs = W.gen_latency_records(900, pods, API, seed=52, background=500)
    kw = dict(latency_limit=20)
    if cpu:
        kw["flags"] = _abi.FLAG_CPU_BACKEND
    parts = [make_engine(pods, SPEC, False, gpu_device, **kw) for _ in range(2)]
    try:
        for r, g in enumerate(parts):
            g.set_apiserver_ips(API)
            sh = D.shard_records(recs, 2, r)
            hb = g.alloc_batch(len(sh.src_ip))
            hb.fill(sh)
            g.submit(hb, len(sh.src_ip))
        before = [g.latency_state() for g in parts]
        assert all(b["capacity_batches"] > 0 and b["capacity_evictions"] > 0 for b in before)
        parts[0].merge_from(parts[1:])
        after, rest = parts[0].latency_state(), parts[1].latency_state()
    finally:
        for g in parts:
            g.close()
    assert after["capacity_evictions"] == sum(b["capacity_evictions"] for b in before)
    assert after["capacity_batches"] == sum(b["capacity_batches"] for b in before)
    assert after["peak_live"] == max(b["peak_live"] for b in before)
    assert rest["capacity_evictions"] == rest["capacity_batches"] == rest["peak_live"] == 0
