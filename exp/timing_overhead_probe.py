"""Probe: C2 step wall time with and without the per-launch HIP timing events (the
bench's timed region records one event per launch on the engine's stream)."""
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

cfg = W.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
pods = W.make_pods(cfg["pods"], seed=cfg["seed"])
n = cfg["records"]
cols, _ = gen_device_records(n, pods, cfg["seed"], torch.device("cuda", 0), dict(cfg["gen"]))
g = GpuAgg(device=0, max_slots=cfg["pods"] + 16, max_ips=2 * cfg["pods"] + 16, sparse_capacity_log2=16)
g.reconcile(W.LOCAL_FWD_DROP)
g.load_endpoints(pods.endpoints)
dc = GpuAgg.device_columns(*cols)
for _ in range(3):
    g.submit_device(dc, n)
g.sync()
for rep in range(3):
    for timing in (False, True):
        g.set_timing(False)
        g.set_timing(timing)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            g.submit_device(dc, n)
        g.sync()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 100
        st = g.stats()
        print(json.dumps({"timing": timing, "ms_per_step": ms, "kernel_ms": st["kernel_ms"] / max(1, st["kernel_launches"])}),
              flush=True)
g.close()
