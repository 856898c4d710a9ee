"""Probe (diagnostics): C5's IP resolution alone -- enrich_kernel over the 10M-record C5
batch (src/dst -> pod slots, HBM radix table) -- next to the C5 aggregation launch."""
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

c5 = W.CONFIGS["c5"]
dev = torch.device("cuda", 0)
pods = W.make_pods(c5["pods"], seed=c5["seed"])
n = c5["records"]
cols, last = gen_device_records(n, pods, c5["seed"], dev, dict(c5["gen"]), chunk=n)
g = GpuAgg(device=0, max_slots=c5["pods"] + 16, max_ips=2 * c5["pods"] + 16, sparse_capacity_log2=23)
g.reconcile(W.C5_SPEC)
g.load_endpoints(pods.endpoints)
for p in last.dns:
    g.dns_intern(p.rcode, p.qtypes, p.query, p.ips, p.num_answers)
dc = GpuAgg.device_columns(*cols)
os_, od = torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev)
for name, fn in (("enrich", lambda: g.enrich_device(dc, n, os_, od)), ("c5_launch", lambda: g.submit_device(dc, n))):
    fn()
    g.sync()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    g.sync()
    print(json.dumps({"probe": name, "records": n, "ms": (time.perf_counter() - t0) / reps * 1e3}), flush=True)
print(json.dumps({"pod_frac_src": float((os_ >= 0).float().mean()), "pod_frac_dst": float((od >= 0).float().mean())}))
g.close()
