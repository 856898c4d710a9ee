"""Sketch-cost ablation for config C3 (diagnostics, not the bench): the C2 metric spec
on 2^27 resident records with no sketch / count-min only / HLL only / both."""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import gen_device_records  # noqa: E402
from retina_amd import GpuAgg  # noqa: E402
from retina_amd import workloads as W  # noqa: E402


def run(name, pods, cols, n, steps=3, **sk):
    g = GpuAgg(device=0, max_slots=len(pods.endpoints) + 16, max_ips=2 * len(pods.endpoints) + 16,
               sparse_capacity_log2=16, **sk)
    g.reconcile(W.LOCAL_FWD_DROP)
    g.load_endpoints(pods.endpoints)
    dc = GpuAgg.device_columns(*cols)
    g.submit_device(dc, n)
    g.sync()
    g.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        g.submit_device(dc, n)
    g.sync()
    wall = (time.perf_counter() - t0) / steps
    st = g.stats()
    g.close()
    ms = st["kernel_ms"] / max(1, st["kernel_launches"])
    print(json.dumps({"variant": name, "records": n, "launch_ms": ms, "wall_ms": wall * 1e3,
                      "kernel": int(st["last_kernel"]), "grec_s": n / ms / 1e6}), flush=True)


def main():
    n = int(os.environ.get("ABLATE_N", 1 << 27))
    pods = W.make_pods(10_000, seed=3)
    cols, _ = gen_device_records(n, pods, 3, torch.device("cuda", 0), {})
    only = set(filter(None, os.environ.get("ABLATE_ONLY", "").split(",")))
    for name, sk in (("none", {}), ("cms", dict(cms_depth=4, cms_width_log2=20)),
                     ("hll", dict(hll_precision=14)),
                     ("both", dict(cms_depth=4, cms_width_log2=20, hll_precision=14))):
        if not only or name in only:
            run(name, pods, cols, n, **sk)


if __name__ == "__main__":
    main()
