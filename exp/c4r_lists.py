"""Probe: c4-remote step time against the wide-key list budget (gpuagg_config.wide_list_mib):
fewer conditional folds with longer lists.  Prints one JSON line per budget."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import gen_device_records  # noqa: E402
from retina_amd import GpuAgg  # noqa: E402
from retina_amd import workloads as W  # noqa: E402

c4 = W.CONFIGS["c4-remote"]
pods = W.make_pods(c4["pods"], seed=c4["seed"])
n = c4["records"]
cols, _ = gen_device_records(n, pods, c4["seed"], torch.device("cuda", 0), dict(c4["gen"]), cache_key="c4-remote")
for mib in [int(x) for x in sys.argv[1:]]:
    g = GpuAgg(device=0, remote_context=True, max_slots=c4["pods"] + 16, max_ips=2 * c4["pods"] + 16,
               sparse_capacity_log2=24, wide_list_mib=mib)
    g.reconcile(W.C1_REMOTE)
    g.load_endpoints(pods.endpoints)
    dc = GpuAgg.device_columns(*cols)
    for _ in range(2):
        g.submit_device(dc, n)
    g.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        g.submit_device(dc, n)
    g.sync()
    ms = (time.perf_counter() - t0) * 100
    g.close()
    print(json.dumps({"wide_list_mib": mib, "ms_per_step": ms, "step_frac": 16 * n / (ms * 1e-3) / 8e12}), flush=True)
