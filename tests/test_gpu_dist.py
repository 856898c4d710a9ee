"""Multi-GPU merge on real device state: two ranks, each with its own GpuAgg
on the GPU, aggregate their 5-tuple shard (dist.shard_of) and merge with
dist.merge_engine -- dense counters, count-min, HLL registers and the sparse group-by table
(remote context + DNS).  Rank 0's series, count-min rows and HLL registers must equal one
engine fed every record; rank 1 must be reset.  The ranks share one GPU, so the collective
backend is gloo (merge_engine stages through host memory); production ranks use RCCL on
distinct GPUs through the same function."""

import os
import queue
import socket
import time

import numpy as np
import pytest

from retina_amd import workloads as W

from .helpers import diff_series, make_engine, to_device

pytestmark = pytest.mark.gpu

SKETCH = dict(cms_depth=4, cms_width_log2=16, hll_precision=10)
LOCAL_SPEC = W.LOCAL_FWD_DROP + W.C5_SPEC
N = 1_500_000


def _data():
    pods = W.make_pods(1_500, seed=21)
    recs = W.gen_records(N, pods, seed=21, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.1,
                         udp_frac=0.15, n_queries=3_000)
    return pods, recs


def _run_engines(pods, recs, device, merge=None):
    """(local+sketch engine, remote engine) fed `recs`; optionally merged."""
    from retina_amd import GpuAgg
    out = []
    for remote, spec, kw in ((False, LOCAL_SPEC, SKETCH), (True, W.C1_REMOTE, {})):
        g = make_engine(pods, spec, remote, device, recs, sparse_capacity_log2=21, **kw)
        if len(recs):
            g.submit_device(GpuAgg.device_columns(*to_device(recs, device)), len(recs))
        g.sync()
        if merge:
            merge(g)
        snap = g.snapshot()
        cms = g.cms_array() if kw else None
        hll = g.hll_array() if kw else None
        g.close()
        out.append((snap, cms, hll))
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from retina_amd import dist as D
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        pods, recs = _data()
        mine = D.shard_records(recs, world, rank)
        res = _run_engines(pods, mine, 0, merge=D.merge_engine)
        q.put((rank, len(mine), res))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, -1, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_engine_merge_equals_single(gpu_device):
    import torch.multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.monotonic() + 240
    while len(res) < world:
        try:
            rank, n, r = q.get(timeout=5)
            assert n >= 0, r
            res[rank] = (n, r)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, "rank exited with %r" % dead
            assert time.monotonic() < deadline, "ranks did not report within 240 s"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] + res[1][0] == N and min(res[0][0], res[1][0]) > 0

    pods, recs = _data()
    want = _run_engines(pods, recs, gpu_device)
    got0, got1 = res[0][1], res[1][1]
    for (ws, wc, wh), (gs, gc, gh), (zs, zc, zh) in zip(want, got0, got1):
        assert gs == ws, diff_series(gs, ws)
        assert not zs, "non-root rank keeps %d series after the merge" % len(zs)
        if wc is not None:
            assert np.array_equal(gc, wc)
            assert np.array_equal(gh, wh)
            assert not zc.any() and not zh.any()
    # the merged state is non-trivial: dense, sparse (DNS, remote) and sketches all present
    assert any(k[0].endswith("dns_request_count") for k in want[0][0])
    assert len(want[1][0]) > 1000 and want[0][1].sum() == 4 * N


LAT_API = [W.ip_le(10, 255, 0, 1), W.ip_le(10, 255, 0, 2)]
LAT_SPEC = [{"metric_name": "node_apiserver_latency"}, {"metric_name": "node_apiserver_handshake_latency"},
            {"metric_name": "node_apiserver_no_response"},
            {"metric_name": "forward_count", "source_labels": ["namespace", "podname"]}]


def _lat_data():
    pods = W.make_pods(200, seed=31)
    return pods, W.gen_latency_records(400, pods, LAT_API, seed=32, background=3000)


def _lat_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from retina_amd import GpuAgg
    from retina_amd import dist as D
    from .test_gpu_latency import _dev
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        pods, recs = _lat_data()
        mine = D.shard_records(recs, world, rank)
        g = make_engine(pods, LAT_SPEC, False, 0)
        g.set_apiserver_ips(LAT_API)
        g.submit_device(GpuAgg.device_columns(*_dev(mine, 0)), len(mine.src_ip))
        D.merge_engine(g)
        st = g.latency_state()
        g.close()
        q.put((rank, len(mine.src_ip), st))
    except Exception as e:
        q.put((rank, -1, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_two_rank_latency_merge(gpu_device):
    """merge_engine sums the node-apiserver latency histograms and no_response of every
    rank into rank 0 before the other ranks reset (their observations used to be lost)."""
    import torch.multiprocessing as mp
    from .latency_helpers import as_state, oracle_latency
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_lat_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.monotonic() + 240
    while len(res) < world:
        try:
            rank, n, r = q.get(timeout=5)
            assert n >= 0, r
            res[rank] = (n, r)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, "rank exited with %r" % dead
            assert time.monotonic() < deadline, "ranks did not report within 240 s"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pods, recs = _lat_data()
    want = as_state(oracle_latency(recs, LAT_API))
    got, rest = res[0][1], res[1][1]
    for k in ("latency_buckets", "latency_count", "latency_sum", "handshake_buckets", "handshake_count",
              "handshake_sum"):
        assert got[k] == want[k], k
    assert got["no_response"] + got["pending"] + rest["pending"] == want["no_response"] + want["pending"]
    assert rest["latency_count"] == 0 and rest["no_response"] == 0
    assert want["latency_count"] > 0


def _nccl_worker(port, q):
    """merge_engine over RCCL (backend "nccl") with one rank: the reduce / all-gather calls
    run on the engine's device memory through __cuda_array_interface__ views, as on an
    8-GPU node; with one rank the merged state must be the engine's own."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from retina_amd import dist as D
    try:
        torch.cuda.set_device(0)  # the device first, then the group (bench.py's order)
        dist.init_process_group("nccl", rank=0, world_size=1)
        pods, recs = _data()
        out = []
        for remote, spec, kw in ((False, LOCAL_SPEC, SKETCH), (True, W.C1_REMOTE, {})):
            from retina_amd import GpuAgg
            g = make_engine(pods, spec, remote, 0, recs, sparse_capacity_log2=21, **kw)
            g.submit_device(GpuAgg.device_columns(*to_device(recs, 0)), len(recs))
            g.sync()
            before = (g.snapshot(), g.cms_array() if kw else None, g.hll_array() if kw else None)
            D.merge_engine(g)
            D.merge_engine(g)  # a second epoch merge: communicators reused
            after = (g.snapshot(), g.cms_array() if kw else None, g.hll_array() if kw else None)
            g.close()
            out.append((before[0] == after[0] and len(before[0]) > 0,
                        kw == {} or (np.array_equal(before[1], after[1]) and np.array_equal(before[2], after[2]))))
        q.put(("ok", out))
    except Exception as e:
        q.put(("err", repr(e)))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_merge_engine_over_rccl_single_rank(gpu_device):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    status, out = q.get(timeout=240)
    p.join(timeout=60)
    assert status == "ok", out
    assert p.exitcode == 0
    assert all(a and b for a, b in out), out
