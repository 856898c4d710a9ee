"""Count-min and HyperLogLog on the GPU at the C3 sketch shape (d=4, w=2^20, p=14).

* state bit-exact against the numpy restatement (oracle/sketch.py), through the
  windowed count-min scatter/fold pass, including list overflow (Zipf-skewed 5-tuples
  push single windows past their list capacity, which falls back to global atomics);
* estimates within the stated bounds (BASELINE.json north_star): count-min never
  under-counts and over-counts by more than eps*N = (e/w)*N for at most delta = e^-d of
  the keys; HLL relative error per pod within 4 sigma, sigma = 1.04/sqrt(2^p).
"""

import math

import numpy as np
import pytest

from oracle import sketch as S
from retina_amd import workloads as W

from .helpers import make_engine, to_device

pytestmark = pytest.mark.gpu

SPEC = [{"metric_name": "forward_count", "source_labels": ["namespace", "podname"]}]


def _run(recs, pods, gpu_device, d=4, w=20, p=14, flags=0):
    from retina_amd import GpuAgg
    g = make_engine(pods, SPEC, False, gpu_device, cms_depth=d, cms_width_log2=w, hll_precision=p, flags=flags)
    try:
        g.submit_device(GpuAgg.device_columns(*to_device(recs, gpu_device)), len(recs))
        g.sync()
        return g.cms_array(), g.hll_array()
    finally:
        g.close()


def _src_slots(pods, src):
    ip_slot = {}
    for s, ep in enumerate(pods.endpoints):
        for ip in ep.ips:
            ip_slot[int(ip)] = s
    lut_ips = np.array(sorted(ip_slot), np.uint32)
    lut_slot = np.array([ip_slot[int(x)] for x in lut_ips], np.int64)
    pos = np.clip(np.searchsorted(lut_ips, src), 0, len(lut_ips) - 1)
    return np.where(lut_ips[pos] == src, lut_slot[pos], -1)


# source lookups through each LDS image form: dense radix (default), radix with its row
# table (FLAG_ROW_RADIX), bucketized cuckoo (FLAG_LDS_CUCKOO)
@pytest.mark.parametrize("flags", [0, 256, 64], ids=["dense-radix", "row-radix", "cuckoo"])
@pytest.mark.parametrize("zipf", [None, 1.2], ids=["uniform", "zipf"])
def test_c3_shape_bit_exact(gpu_device, zipf, flags):
    pods = W.make_pods(200, seed=41)
    recs = W.gen_records(3_000_000, pods, seed=42, udp_frac=0.2, zipf=zipf)
    if zipf:  # heavy 5-tuples: repeat a few flows so some count-min windows overflow
        hot = np.random.default_rng(1).integers(0, 64, len(recs)) == 0
        recs.dst_ip[hot] = recs.dst_ip[0]
        recs.src_ip[hot] = recs.src_ip[0]
        recs.ports[hot] = recs.ports[0]
    cms, hll = _run(recs, pods, gpu_device, flags=flags)
    want = np.zeros((4, 1 << 20), np.uint32)
    S.cms_update(want, recs.src_ip, recs.dst_ip, recs.ports, recs.meta & np.uint32(0xFF))
    assert np.array_equal(cms, want)
    want_h = np.zeros((len(pods.endpoints), 1 << 14), np.uint8)
    S.hll_update(want_h, _src_slots(pods, recs.src_ip), recs.dst_ip, 14)
    assert np.array_equal(hll[:len(pods.endpoints)], want_h)


def test_count_min_bounds(gpu_device):
    pods = W.make_pods(500, seed=43)
    recs = W.gen_records(4_000_000, pods, seed=44, udp_frac=0.2, zipf=1.2)
    cms, _ = _run(recs, pods, gpu_device)
    key = np.stack([recs.src_ip, recs.dst_ip, recs.ports, recs.meta & np.uint32(0xFF)], 1)
    uniq, true = np.unique(key, axis=0, return_counts=True)
    est = S.cms_estimate(cms, uniq[:, 0], uniq[:, 1], uniq[:, 2], uniq[:, 3])
    assert (est >= true).all()                      # count-min never under-counts
    n, eps, delta = len(recs), math.e / (1 << 20), math.exp(-4)
    frac_bad = float(np.mean(est - true > eps * n))
    assert frac_bad <= delta, (frac_bad, delta)


def test_hll_relative_error(gpu_device):
    pods = W.make_pods(40, seed=45, secondary_frac=0.0)
    n = 4_000_000
    rng = np.random.default_rng(46)
    recs = W.gen_records(n, pods, seed=46, pod_frac=1.0)
    recs.dst_ip[:] = rng.integers(1, 1 << 32, n, dtype=np.uint64).astype(np.uint32)  # ~distinct dsts
    _, hll = _run(recs, pods, gpu_device)
    slot = _src_slots(pods, recs.src_ip)
    sigma = 1.04 / math.sqrt(1 << 14)
    errs = []
    for s in range(len(pods.endpoints)):
        true = len(np.unique(recs.dst_ip[slot == s]))
        if true < 10_000:
            continue
        errs.append(abs(S.hll_estimate(hll[s]) - true) / true)
    assert len(errs) >= 30
    assert max(errs) <= 4 * sigma, max(errs)
    assert float(np.mean(errs)) <= 1.5 * sigma


def test_c3_full_shape_bit_exact(gpu_device):
    """BASELINE.json config 3 at its benched per-GPU shape: 10k pods (HLL 10k x 16 KiB =
    160 MiB), count-min d=4 w=2^20, 2^27 records drawn from SURVEY.md 8d's flow
    distribution (10^7 flows, src in the pods, dst among 10^6 IPs), C2's metrics beside the
    sketches.  Count-min rows, HLL registers and every series bit-exact against the numpy
    restatements, accumulated chunk by chunk on the host."""
    import torch
    from oracle.vectorized import LocalDense
    from retina_amd import GpuAgg
    cfg = W.CONFIGS["c3"]
    pods = W.make_pods(cfg["pods"], seed=cfg["seed"])
    n, chunk = 1 << 27, 1 << 23
    g = make_engine(pods, W.LOCAL_FWD_DROP, False, gpu_device, cms_depth=4, cms_width_log2=20,
                    hll_precision=14)
    dev = torch.device("cuda", gpu_device)
    cols = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(6)]
    want_c = np.zeros((4, 1 << 20), np.uint32)
    want_h = np.zeros((len(pods.endpoints), 1 << 14), np.uint8)
    v = LocalDense(W.LOCAL_FWD_DROP, pods.endpoints)
    for k in range(n // chunk):
        r = W.gen_records(chunk, pods, seed=3000 + k, **cfg["gen"])
        for t, a in zip(cols, (r.src_ip, r.dst_ip, r.bytes, r.meta, r.ports, r.dns_id)):
            t[k * chunk:(k + 1) * chunk].copy_(torch.from_numpy(a.view(np.int32)))
        S.cms_update(want_c, r.src_ip, r.dst_ip, r.ports, r.meta & np.uint32(0xFF))
        S.hll_update(want_h, _src_slots(pods, r.src_ip), r.dst_ip, 14)
        v.add(r)
    try:
        g.submit_device(GpuAgg.device_columns(*cols), n)
        got = g.snapshot()
        cms, hll = g.cms_array(), g.hll_array()
    finally:
        g.close()
    del cols
    assert got == v.series()
    assert np.array_equal(cms, want_c)
    assert np.array_equal(hll[:len(pods.endpoints)], want_h)
    assert int(cms[0].sum()) == n


@pytest.mark.parametrize("flags", [0, 8], ids=["deferred", "per-batch"])
def test_deferred_sketch_folds_exact(gpu_device, flags):
    """Small launches (the Go plugin's batch geometry) defer their count-min / HLL folds:
    the scatters append to one set of lists sized for 2^22 records per workgroup and
    fold_pending folds them once.  Exact against the restatement across mid-stream reads
    (cms_array / hll_array fold what waits), 1026 launches of 2^20 records (the 1024-launch
    budget overflows and folds; the batch is resubmitted, so count-min is linear in the
    repeats and HLL idempotent), ragged launches and a slot-table growth (relayout folds).
    FLAG_FOLD_PER_BATCH (8) keeps per-launch folds as the reference point."""
    from retina_amd import GpuAgg
    pods = W.make_pods(300, seed=51)
    more = W.make_pods(900, seed=51)  # same IPs for the first 300: the slot table grows
    g = make_engine(pods, W.LOCAL_FWD_DROP, False, gpu_device, cms_depth=4, cms_width_log2=16,
                    hll_precision=12, flags=flags, max_slots=2048, max_ips=4096)
    want_c = np.zeros((4, 1 << 16), np.uint32)
    want_h = np.zeros((len(more.endpoints), 1 << 12), np.uint8)

    def expect(r, src_pods, times=1):
        one = np.zeros_like(want_c)
        S.cms_update(one, r.src_ip, r.dst_ip, r.ports, r.meta & np.uint32(0xFF))
        want_c[:] += one * np.uint32(times)
        S.hll_update(want_h, _src_slots(src_pods, r.src_ip), r.dst_ip, 12)

    def check(tag):
        assert np.array_equal(g.cms_array(), want_c), tag
        h = g.hll_array()  # rows of the slots in use (grown with them)
        n = min(len(h), len(want_h))
        assert np.array_equal(h[:n], want_h[:n]) and not want_h[n:].any(), tag

    total = 0
    try:
        for k in range(6):  # distinct small batches, ragged sizes
            m = (1 << 16) + 1000 * k + k
            r = W.gen_records(m, pods, seed=5200 + k, udp_frac=0.2)
            g.submit_device(GpuAgg.device_columns(*to_device(r, gpu_device)), m)
            expect(r, pods)
            total += m
        check("after 6 small launches")
        big = W.gen_records(1 << 20, pods, seed=5300, udp_frac=0.2)
        cols = GpuAgg.device_columns(*to_device(big, gpu_device))
        for _ in range(1026):
            g.submit_device(cols, 1 << 20)
        expect(big, pods, 1026)
        total += 1026 << 20
        check("after 1026 launches of 2^20")
        g.load_endpoints(more.endpoints[len(pods.endpoints):], version=2)
        for k in range(3):
            r = W.gen_records(50_000, more, seed=5400 + k, udp_frac=0.2)
            g.submit_device(GpuAgg.device_columns(*to_device(r, gpu_device)), 50_000)
            expect(r, more)
            total += 50_000
            if k == 0:
                g.load_endpoints([], version=3)  # a commit between launches
        g.sync()
        check("final")
        assert g.stats()["records"] == total
    finally:
        g.close()
