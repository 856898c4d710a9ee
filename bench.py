"""Benchmark: flow records/s aggregated on MI355X (BASELINE.json metric).

Workload (config C2): a 100M-record batch of synthetic decoded flows,
10k pods, local context, per-pod forward count/bytes + drop-reason histogram
(forward_count, forward_bytes, drop_count, drop_bytes with sourceLabels
[namespace, podname]).  One step = one aggregation pass over the whole batch, with
the records already resident in HBM.  Weak scaling: every rank aggregates its own
100M-record shard; the counters are merged once per timed region with an RCCL
all-reduce (the per-scrape-epoch merge).

    python bench.py [--gpus N --steps K --warmup W --config c2 --records R]
"""

from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "flow records/sec aggregated (node, 1/2/4/8 GPU); % of HBM peak GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_RECORD = 16  # src_ip, dst_ip, bytes, meta


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class _CAI:
    """__cuda_array_interface__ view of a raw device pointer (for RCCL merges)."""

    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}


def device_view(ptr: int, n: int, typestr: str, device):
    import torch
    return torch.as_tensor(_CAI(ptr, n, typestr), device=device)


def gen_device_records(n: int, pods, seed: int, device, gen_kw, chunk: int = 8_000_000):
    """Generates the workload on the host in chunks and keeps it resident in HBM."""
    import torch
    from retina_amd import workloads as W
    cols = [torch.empty(n, dtype=torch.int32, device=device) for _ in range(6)]
    start, k = 0, 0
    while start < n:
        m = min(chunk, n - start)
        r = W.gen_records(m, pods, seed * 1000 + k, **gen_kw)
        for t, a in zip(cols, (r.src_ip, r.dst_ip, r.bytes, r.meta, r.ports, r.dns_id)):
            t[start:start + m].copy_(torch.from_numpy(a.view(np.int32)))
        start += m
        k += 1
    return cols, r


def cpu_baseline(cfg_name: str, pods, spec, sample: int, seed: int, gen_kw):
    """The C port of the reference path (oracle/ref_cpu.c, go-shaped: dotted-string IPs,
    string-keyed cache and label maps; enrich + every ProcessFlow per flow on one thread)
    timed on a bounded sample of the same workload."""
    from oracle.ref_cpu import RefCPU
    from retina_amd import workloads as W
    recs = W.gen_records(sample, pods, seed, **gen_kw)
    r = RefCPU(spec, pods.endpoints, False, recs.dns)
    dt = r.process(recs)
    r.close()
    return {"value": sample / dt, "unit": "records/s", "cores": 1, "kind": "port",
            "sample": "%d records of config %s through oracle/ref_cpu.c (C port of enricher.go + "
                      "metrics module, 1 thread), %.1f s" % (sample, cfg_name, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--records", type=int, default=0, help="records per GPU (default: config size)")
    ap.add_argument("--cpu-sample", type=int, default=12_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from retina_amd import GpuAgg, _abi
    from retina_amd import workloads as W

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)

    cfg = W.CONFIGS[args.config]
    n = args.records or cfg["records"]
    gen_kw = dict(cfg["gen"])
    spec = W.LOCAL_FWD_DROP
    pods = W.make_pods(cfg["pods"], seed=cfg["seed"])
    t0 = time.time()
    cols, _ = gen_device_records(n, pods, cfg["seed"] + 7919 * rank, device, gen_kw)
    torch.cuda.synchronize()
    log("rank %d: %d records resident in HBM (%.1f s)" % (rank, n, time.time() - t0))

    g = GpuAgg(device=local_rank, remote_context=False, max_slots=cfg["pods"] + 16,
               max_ips=2 * cfg["pods"] + 16, sparse_capacity_log2=16)
    g.reconcile(spec)
    g.load_endpoints(pods.endpoints)
    dcols = GpuAgg.device_columns(*cols)

    for _ in range(args.warmup):
        g.submit_device(dcols, n)
    g.sync()

    st = g.state()
    dense_cnt = dense_byt = None
    if world > 1:
        dense_cnt = device_view(st.dense_count, st.dense_len, "<i8", device)
        dense_byt = device_view(st.dense_bytes, st.dense_len, "<i8", device)

    # ---- timed region --------------------------------------------------------------
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    g.set_timing(False)
    g.set_timing(True)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        g.submit_device(dcols, n)
    g.sync()
    if world > 1:  # per-epoch merge over RCCL/xGMI: sum of u64 counters
        dist.all_reduce(dense_cnt)
        dist.all_reduce(dense_byt)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    stats = g.stats()
    g.set_timing(False)
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    kernel_ms = stats["kernel_ms"] / max(1, stats["kernel_launches"])
    fold_ms = stats["fold_ms"] / max(1, stats["kernel_launches"])
    achieved = BYTES_PER_RECORD * n / (kernel_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch_corrected")
        except Exception:
            traffic = None

    result = {
        "metric": METRIC,
        "value": n * world * args.steps / elapsed,
        "unit": "records/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {
            "workload": "C2: %d-record batch per GPU, %d pods, local context, per-pod "
                        "forward count/bytes + drop-reason histogram [namespace, podname]"
                        % (n, cfg["pods"]),
            "records_per_gpu": n,
            "pods": cfg["pods"],
            "metrics": [s["metric_name"] for s in spec],
            "parallelism": "dp%d (records sharded, counters all-reduced once per timed region)" % world,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": _abi.KERNEL_NAMES.get(int(stats["last_kernel"])),
            "kernel_ms": kernel_ms,
            "other_kernels_ms": fold_ms,
            "bytes_per_record": BYTES_PER_RECORD,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.config, pods, spec, args.cpu_sample, cfg["seed"], gen_kw)
    g.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
