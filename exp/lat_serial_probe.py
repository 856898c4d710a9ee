"""Probe: cost of a capacity-bound node-apiserver latency batch at the Go
plugin's 2^20 records.  When the live requests pass the ttlcache LIMIT, lat_serial_kernel
replays the batch's events on one GPU thread; the serial pass's cost grows with the events,
not with the limit, so a small latency_limit forces it on an ordinary batch.  Prints the
per-batch wall time with the capacity bound (limit 1000) and not bound (limit 100000)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from retina_amd import GpuAgg  # noqa: E402
from retina_amd import workloads as W  # noqa: E402

API = [W.ip_le(10, 255, 0, 1), W.ip_le(10, 255, 0, 2)]
SPEC = [{"metric_name": "node_apiserver_latency"}, {"metric_name": "node_apiserver_handshake_latency"},
        {"metric_name": "node_apiserver_no_response"}]
pods = W.make_pods(1000, seed=61)
recs = W.gen_latency_records(110_000, pods, API, seed=62, background=150_000)
n = min(len(recs.src_ip), 1 << 20)
for limit in (100_000, 1000):
    g = GpuAgg(device=0, max_slots=1100, max_ips=2200, latency_limit=limit)
    g.reconcile(SPEC)
    g.load_endpoints(pods.endpoints)
    g.set_apiserver_ips(API)
    hb = g.alloc_batch(n)
    hb.fill(recs)
    g.submit(hb, n)  # warm-up (allocations)
    g.sync()
    g.reset()
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        g.submit(hb, n)
        g.sync()
        times.append((time.perf_counter() - t0) * 1e3)
    st = g.latency_state()
    print(json.dumps({"limit": limit, "records": n, "events": int(st["latency_count"] + st["no_response"]),
                      "ms_per_batch": times, "capacity_batches": st["capacity_batches"],
                      "peak_live": st["peak_live"]}), flush=True)
    g.close()
