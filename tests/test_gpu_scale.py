"""GPU parity at larger sizes: against the C port (millions of records) and, at the full
BASELINE.json C2 size (100M records), against the numpy restatement -- exact, plus
size-independent properties (determinism, host-fed == device-resident, chunking)."""

import numpy as np
import pytest

from oracle.ref_cpu import RefCPU, values_only
from oracle.vectorized import LocalDense
from retina_amd import workloads as W

from .helpers import diff_series, engine_series, make_engine

pytestmark = pytest.mark.gpu

MID = [
    ("c1-local", W.C1_LOCAL, False, 10_000, {}),
    ("c1-remote", W.C1_REMOTE, True, 10_000, {}),
    ("c2-local", W.LOCAL_FWD_DROP, False, 10_000, {}),
    ("c2-local-lds-cuckoo", W.LOCAL_FWD_DROP, False, 10_000, {"flags": 64}),  # FLAG_LDS_CUCKOO
    ("c2-local-row-radix", W.LOCAL_FWD_DROP, False, 10_000, {"flags": 256}),  # FLAG_ROW_RADIX
    ("c4-zipf", W.LOCAL_FWD_DROP, False, 10_000, {"zipf": 1.2}),
    ("c4-flows", W.LOCAL_FWD_DROP, False, 10_000, dict(W.CONFIGS["c4"]["gen"])),
    ("c4-flows-remote", W.C1_REMOTE, True, 10_000, dict(W.CONFIGS["c4"]["gen"])),
    ("c5-local", W.C5_SPEC, False, 100_000, {"drop_frac": 0.0, "retrans_frac": 0.05, "dns_frac": 0.35}),
]


@pytest.mark.parametrize("cid,sp,remote,npods,gen", MID, ids=[m[0] for m in MID])
def test_midsize_vs_c_port(gpu_device, cid, sp, remote, npods, gen):
    gen = dict(gen)
    flags = gen.pop("flags", 0)
    pods = W.make_pods(npods, seed=2)
    recs = W.gen_records(1_000_000, pods, seed=77, **gen)
    r = RefCPU(sp, pods.endpoints, remote, recs.dns)
    r.process(recs)
    want = r.series()
    r.close()
    got = values_only(engine_series(recs, pods, sp, remote, gpu_device, host_fed=False, chunks=3,
                                    sparse_capacity_log2=23, flags=flags))
    assert got == want, diff_series(got, want)


def test_full_c2_exact(gpu_device):
    """BASELINE.json config 2 at full size: 100M records, 10k pods, 1 MI355X."""
    import torch
    from retina_amd import GpuAgg
    pods = W.make_pods(10_000, seed=2)
    n, chunk = 100_000_000, 10_000_000
    g = make_engine(pods, W.LOCAL_FWD_DROP, False, gpu_device)
    v = LocalDense(W.LOCAL_FWD_DROP, pods.endpoints)
    dev = torch.device("cuda", gpu_device)
    cols = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(6)]
    for k in range(n // chunk):
        r = W.gen_records(chunk, pods, seed=1000 + k)
        v.add(r)
        for t, a in zip(cols, (r.src_ip, r.dst_ip, r.bytes, r.meta, r.ports, r.dns_id)):
            t[k * chunk:(k + 1) * chunk].copy_(torch.from_numpy(a.view(np.int32)))
    dc = GpuAgg.device_columns(*cols)
    g.submit_device(dc, n)
    got = g.snapshot()
    want = v.series()
    assert got == want, diff_series(got, want)
    # determinism: a second pass doubles every series exactly
    g.submit_device(dc, n)
    got2 = g.snapshot()
    assert got2 == {k: 2 * x for k, x in got.items()}
    g.close()


def test_host_fed_equals_device_and_chunking(gpu_device):
    pods = W.make_pods(2_000, seed=3)
    recs = W.gen_records(3_000_000, pods, seed=3, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.1,
                         udp_frac=0.1, n_queries=2000)
    sp = W.LOCAL_FWD_DROP + W.C5_SPEC
    a = engine_series(recs, pods, sp, False, gpu_device, host_fed=True, chunks=1)
    b = engine_series(recs, pods, sp, False, gpu_device, host_fed=False, chunks=7)
    assert a == b, diff_series(a, b)


@pytest.mark.parametrize("flags", [0, 256, 64, 1],
                         ids=["tier1-dense-radix", "tier1-row-radix", "tier1-cuckoo", "no-lds-ip-table"])
def test_packed_field_overflow_exact(gpu_device, flags):
    """Packed LDS counters (u32 count:12|bytes:20 in tier-1, u64 count:20|bytes:44 in the
    other kernels and the fold windows) must carry exactly.  One hot pod pair, 60M
    records: LDS count fields wrap many times, byte fields carry, packets >= 2^20 / 2^24
    bytes take the global path, and the hot drop bins overflow their spill lists into
    global atomics.  Expected = a 10-record batch x 6M (linearity)."""
    import torch
    from retina_amd import GpuAgg
    pods = W.make_pods(10_000, seed=5)
    base = W.gen_records(400, pods, seed=5, pod_frac=1.0, drop_frac=0.5)
    verdict = (base.meta >> 8) & 0xFF
    ok = (base.src_ip != base.dst_ip)
    f = int(np.flatnonzero((verdict == W.V_FWD) & ok)[0])
    d = int(np.flatnonzero((verdict == W.V_DROP) & ok)[0])
    idx = np.array([f, f, f] + [d] * 7)
    # (the last drop exceeds the 29-bit byte field of the tier-1 drop queue: added at the push)
    nbytes = np.array([1_000_000, (1 << 20) - 1, 5_000_000] + [(1 << 24) - 1] * 5 + [20_000_000, (1 << 31) + 5],
                      np.uint32)
    ten = W.Records(base.src_ip[idx], base.dst_ip[idx], nbytes, base.meta[idx], base.ports[idx],
                    base.dns_id[idx])
    reps = 6_000_000
    v = LocalDense(W.LOCAL_FWD_DROP, pods.endpoints)
    v.add(ten)
    want = {k: x * reps for k, x in v.series().items()}
    dev = torch.device("cuda", gpu_device)
    cols = [torch.from_numpy(np.tile(a, reps).view(np.int32)).to(dev)
            for a in (ten.src_ip, ten.dst_ip, ten.bytes, ten.meta, ten.ports, ten.dns_id)]
    g = make_engine(pods, W.LOCAL_FWD_DROP, False, gpu_device, flags=flags)
    g.submit_device(GpuAgg.device_columns(*cols), len(ten) * reps)
    got = g.snapshot()
    g.close()
    del cols
    assert got == want, diff_series(got, want)


DEFER = [
    ("c2", W.LOCAL_FWD_DROP, False, 10_000, {}),
    ("c5", W.C5_SPEC, False, 100_000, {"drop_frac": 0.0, "retrans_frac": 0.05, "dns_frac": 0.35}),
    # wide (192-bit) keys through the per-segment lists: local ip option and remote context
    ("c1-local", W.C1_LOCAL, False, 10_000, {}),
    ("c4-remote", W.C1_REMOTE, True, 10_000, dict(W.CONFIGS["c4"]["gen"])),
]


@pytest.mark.parametrize("cid,sp,remote,npods,gen", DEFER, ids=[d[0] for d in DEFER])
def test_deferred_folds_exact(gpu_device, cid, sp, remote, npods, gen):
    """Spill / segment lists of consecutive launches are folded once (gpuagg_sync or any
    state read).  143 batches of unequal sizes: a growing chunk changes the list geometry,
    a snapshot folds early, then 136 equal batches exhaust the 64-launch budget twice --
    every case equals the C port and the engine folding after each batch."""
    from retina_amd import GpuAgg, _abi
    from .helpers import to_device
    pods = W.make_pods(npods, seed=8)
    recs = W.gen_records(2_000_000, pods, seed=81, **gen)
    sizes = [30_000, 30_000, 250_000, 20_000] + [6_800] * 136 + [400_000, 10_007, 333_333]
    bounds = np.concatenate([[0], np.cumsum(sizes)])
    assert bounds[-1] <= len(recs)
    n_mid, n = int(bounds[4]), int(bounds[-1])

    def run(flags):
        g = make_engine(pods, sp, remote, gpu_device, recs, sparse_capacity_log2=23, flags=flags)
        try:
            ts = to_device(recs, gpu_device)
            mid = None
            for k, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
                g.submit_device(GpuAgg.device_columns(*[x[int(a):] for x in ts]), int(b - a))
                if k == 3:  # then 136 equal batches: more than kDeferLaunches (64) per budget
                    mid = g.snapshot()
            return mid, g.snapshot()
        finally:
            g.close()

    def port(m):
        part = W.Records(recs.src_ip[:m], recs.dst_ip[:m], recs.bytes[:m], recs.meta[:m], recs.ports[:m],
                         recs.dns_id[:m])
        r = RefCPU(sp, pods.endpoints, remote, recs.dns)
        r.process(part)
        s = r.series()
        r.close()
        return s

    mid, end = run(0)
    mid1, end1 = run(_abi.FLAG_FOLD_PER_BATCH)
    assert mid == mid1 and end == end1
    want_mid, want = port(n_mid), port(n)
    assert values_only(mid) == want_mid, diff_series(values_only(mid), want_mid)
    assert values_only(end) == want, diff_series(values_only(end), want)


@pytest.mark.parametrize("gen", [dict(W.CONFIGS["c4"]["gen"]), {"flows": 64, "flow_zipf": 1.2, "n_dst": 64}],
                         ids=["zipf-1e7-flows", "64-flows"])
def test_hot_key_cache_exact(gpu_device, gen):
    """The LDS hot-key cache in front of the group-by table (remote context, C4's Zipf
    flows and a 64-flow extreme where every key is hot in every workgroup) equals the
    table-only path and the C port."""
    from retina_amd import _abi
    pods = W.make_pods(10_000, seed=9)
    recs = W.gen_records(1_500_000, pods, seed=91, **gen)
    a = values_only(engine_series(recs, pods, W.C1_REMOTE, True, gpu_device, host_fed=False, chunks=2,
                                  sparse_capacity_log2=23))
    b = values_only(engine_series(recs, pods, W.C1_REMOTE, True, gpu_device, host_fed=False, chunks=2,
                                  sparse_capacity_log2=23, flags=_abi.FLAG_NO_HOT_KEYS))
    assert a == b, diff_series(a, b)
    # neither the hot-key cache nor the per-segment lists: memory-side atomics only
    c = values_only(engine_series(recs, pods, W.C1_REMOTE, True, gpu_device, host_fed=False, chunks=2,
                                  sparse_capacity_log2=23,
                                  flags=_abi.FLAG_NO_HOT_KEYS | _abi.FLAG_NO_WIDE_LISTS))
    assert a == c, diff_series(a, c)
    # C1_REMOTE has no port / DNS labels: the 24-byte list entries (FLAG_NARROW_ENTRIES)
    # agree with the default 32-byte ones
    d = values_only(engine_series(recs, pods, W.C1_REMOTE, True, gpu_device, host_fed=False, chunks=2,
                                  sparse_capacity_log2=23, flags=_abi.FLAG_NARROW_ENTRIES))
    assert a == d, diff_series(a, d)
    r = RefCPU(W.C1_REMOTE, pods.endpoints, True, recs.dns)
    r.process(recs)
    want = r.series()
    r.close()
    assert a == want, diff_series(a, want)


def _table_entries(g, device):
    """The engine's group-by table as canonical (k0, k1, k2) -> (count, bytes) tensors:
    exported on the device, keys that took two slots summed (torch.unique + index_add)."""
    import torch
    st = g.state()
    cap = int(st.sparse_len)
    out = torch.empty((cap, 5), dtype=torch.int64, device=device)
    n = g.sparse_export(out.data_ptr(), cap)
    e = out[:n]
    keys, inv = torch.unique(e[:, :3], dim=0, return_inverse=True)
    vals = torch.zeros((keys.shape[0], 2), dtype=torch.int64, device=device)
    vals.index_add_(0, inv, e[:, 3:5])
    return keys, vals


@pytest.mark.parametrize("flags", [0, 512], ids=["32-byte-entries", "24-byte-entries"])
def test_one_new_key_many_lanes(gpu_device, flags):
    """A handful of flows, no LDS hot-key cache: every update is a list entry, so the
    wide fold's balanced lanes meet long runs of the same new key at once.  Each key must
    take exactly one table slot (the probe waits while a lane publishes it, instead of
    claiming the next slot), nothing may be dropped, and the series equal the C port."""
    import torch
    from retina_amd import _abi
    pods = W.make_pods(10_000, seed=12)
    recs = W.gen_records(2_000_000, pods, seed=121, flows=4, flow_zipf=None, n_dst=4)
    g = make_engine(pods, W.C1_REMOTE, True, gpu_device, sparse_capacity_log2=20,
                    flags=_abi.FLAG_NO_HOT_KEYS | flags)
    try:
        from .helpers import to_device
        from retina_amd import GpuAgg
        ts = to_device(recs, gpu_device)
        half = len(recs) // 2
        for a, b in ((0, half), (half, len(recs))):
            g.submit_device(GpuAgg.device_columns(*[x[a:] for x in ts]), b - a)
        g.sync()
        assert g.stats()["sparse_dropped"] == 0
        st = g.state()
        cap = int(st.sparse_len)
        out = torch.empty((cap, 5), dtype=torch.int64, device=torch.device("cuda", gpu_device))
        n = g.sparse_export(out.data_ptr(), cap)
        keys = out[:n, :3]
        assert torch.unique(keys, dim=0).shape[0] == n  # one slot per key
        got = values_only(g.snapshot())
    finally:
        g.close()
    r = RefCPU(W.C1_REMOTE, pods.endpoints, True, recs.dns)
    r.process(recs)
    want = r.series()
    r.close()
    assert got == want, diff_series(got, want)


def test_full_c4_remote_linearity(gpu_device):
    """C4 through the remote context at the full bench size: 100M Zipf(1.2) flow records,
    every update a 192-bit group-by key (~6.7M distinct).  The per-segment lists + LDS
    segment folds equal the memory-side-atomics path exactly; a second pass of the same
    records doubles every entry (determinism, linearity); no update is dropped."""
    import torch
    from retina_amd import GpuAgg, _abi
    pods = W.make_pods(10_000, seed=4)
    n, chunk = 100_000_000, 8_000_000
    dev = torch.device("cuda", gpu_device)
    cols = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(6)]
    for k, a in enumerate(range(0, n, chunk)):
        m = min(chunk, n - a)
        r = W.gen_records(m, pods, seed=4000 + k, **W.CONFIGS["c4"]["gen"])
        for t, x in zip(cols, (r.src_ip, r.dst_ip, r.bytes, r.meta, r.ports, r.dns_id)):
            t[a:a + m].copy_(torch.from_numpy(x.view(np.int32)))
    dc = GpuAgg.device_columns(*cols)
    g = make_engine(pods, W.C1_REMOTE, True, gpu_device, sparse_capacity_log2=24)
    g.submit_device(dc, n)
    g.sync()
    k1, v1 = _table_entries(g, dev)
    g.submit_device(dc, n)
    g.sync()
    k2, v2 = _table_entries(g, dev)
    assert g.stats()["sparse_dropped"] == 0
    g.close()
    assert torch.equal(k1, k2) and torch.equal(v2, 2 * v1)
    assert int(v1[:, 0].sum()) == n  # every record is one forward or one drop update
    b = make_engine(pods, W.C1_REMOTE, True, gpu_device, sparse_capacity_log2=24,
                    flags=_abi.FLAG_NO_HOT_KEYS | _abi.FLAG_NO_WIDE_LISTS)
    b.submit_device(dc, n)
    b.sync()
    kb, vb = _table_entries(b, dev)
    b.close()
    assert torch.equal(k1, kb) and torch.equal(v1, vb)
