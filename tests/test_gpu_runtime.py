"""Runtime properties of the engine on the GPU: one HIP runtime per process, and the
double-buffered host-fed submit (include/gpuagg.h: gpuagg_submit returns once the batch's
H2D copies are done, while its aggregation still runs)."""

import numpy as np
import pytest

from retina_amd import workloads as W

from .helpers import diff_series, engine_series, make_engine

pytestmark = pytest.mark.gpu


def test_single_hip_runtime_mapped(gpu_device):
    """torch and libgpuagg.so share one libamdhip64 / libhsa-runtime64 (retina_amd/_abi.py)."""
    import torch
    from retina_amd import _abi
    pods = W.make_pods(50, seed=1)
    g = make_engine(pods, W.LOCAL_FWD_DROP, False, gpu_device)
    t = torch.ones(1024, device=torch.device("cuda", gpu_device))
    torch.cuda.synchronize()
    maps = _abi.hip_runtimes_mapped()
    g.close()
    assert float(t.sum()) == 1024.0
    assert len(maps["libamdhip64"]) == 1, maps
    assert len(maps["libhsa-runtime64"]) == 1, maps


def test_double_buffered_host_submit(gpu_device):
    """Two pinned batches, filled alternately while the previous batch aggregates: the
    series equal the device-resident run, and submits return before their aggregation
    has finished (the copy of batch k+1 overlaps the kernels of batch k)."""
    pods = W.make_pods(2_000, seed=7)
    recs = W.gen_records(6_000_000, pods, seed=7, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.05,
                         udp_frac=0.1, n_queries=500)
    sp = W.LOCAL_FWD_DROP + W.C5_SPEC
    want = engine_series(recs, pods, sp, False, gpu_device, host_fed=False)
    g = make_engine(pods, sp, False, gpu_device, recs)
    try:
        cap = 500_000
        batches = [g.alloc_batch(cap), g.alloc_batch(cap)]
        for k, start in enumerate(range(0, len(recs), cap)):
            hb = batches[k & 1]
            n = hb.fill(recs, start)
            g.submit(hb, n)
        got = g.snapshot()
        st = g.stats()
    finally:
        g.close()
    assert got == want, diff_series(got, want)
    assert st["batches"] == 12 and st["records"] == len(recs)
    assert st["async_returns"] > 0, st


def test_raw_host_submit_double_buffered(gpu_device):
    """gpuagg_submit_raw over many host chunks equals one device-resident raw submit."""
    import torch
    pods = W.make_pods(1_000, seed=9)
    raw = W.gen_raw_packets(2_000_000, pods, seed=9, udp_frac=0.1)
    sp = W.LOCAL_FWD_DROP + W.C5_SPEC[:1]
    a = make_engine(pods, sp, False, gpu_device)
    b = make_engine(pods, sp, False, gpu_device)
    try:
        a.submit_raw(1, raw, chunk=150_000)
        dev = torch.from_numpy(raw.view(np.int32)).to(torch.device("cuda", gpu_device))
        b.submit_raw_device(1, dev.data_ptr(), len(raw) // 72)
        b.sync()
        ga, gb = a.snapshot(), b.snapshot()
    finally:
        a.close()
        b.close()
    assert ga == gb, diff_series(ga, gb)
    assert sum(ga.values()) > 0
