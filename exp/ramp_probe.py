"""Probe: per-launch C2 kernel time (HIP events) for 60 launches after the host-side data
generation, then again after 2 s idle: is there a warm-up ramp (clocks) the bench's 5
warm-up steps do not cover?"""
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

cfg = W.CONFIGS["c2"]
pods = W.make_pods(cfg["pods"], seed=cfg["seed"])
n = cfg["records"]
cols, _ = gen_device_records(n, pods, cfg["seed"], torch.device("cuda", 0), dict(cfg["gen"]))
g = GpuAgg(device=0, max_slots=cfg["pods"] + 16, max_ips=2 * cfg["pods"] + 16, sparse_capacity_log2=16)
g.reconcile(W.LOCAL_FWD_DROP)
g.load_endpoints(pods.endpoints)
dc = GpuAgg.device_columns(*cols)
g.set_timing(True)
for phase in ("after_gen", "after_idle_2s"):
    ks = []
    t0 = time.perf_counter()
    for i in range(60):
        g.set_timing(False)
        g.set_timing(True)
        g.submit_device(dc, n)
        g.sync()
        st = g.stats()
        ks.append(round(st["kernel_ms"], 4))
    print(json.dumps({"phase": phase, "kernel_ms": ks, "wall_ms_per_launch": (time.perf_counter() - t0) / 60 * 1e3}),
          flush=True)
    time.sleep(2)
g.close()
