"""Ablation timings of the aggregation launch on one MI355X (diagnostics, not the bench).

Runs the same resident 100M-record C2 batch through metric specs of increasing cost and
prints one JSON line per variant with the HIP-event time per launch:
  none      no metric groups: record loads + IP probes only
  fwd       forward_count/bytes (dense, fully in LDS)
  drop      drop_count/bytes    (dense, LDS window + spill lists + fold)
  c2        forward + drop      (the bench spec)
  c2-1kpods C2 spec with 1k pods (every dense bin in LDS, no spill)
  c4-zipf   C2 spec on C4's Zipf(1.2) records (LDS atomic contention)
  *-hbm-ip-table  same with FLAG_NO_LDS_IP_TABLE (IP table in HBM, u64 LDS bins)
  remote    C1 remote spec (sparse table)
  c5*       C5 batch (100k pods) with the C5 spec, and with each of its metrics alone
  c2-lat    C2 spec + node-apiserver latency metrics (the join's filter pass over 100M rows)
  raw-packet  decode of 72-byte packetparser records (C2 columns re-encoded) + C2 forward
              aggregation; decode_ms is the decode kernel, 92 B/record of HBM traffic
"""

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

FWD = W.LOCAL_FWD_DROP[:2]
DROP = W.LOCAL_FWD_DROP[2:]


ONLY = set(filter(None, os.environ.get("ABLATE_ONLY", "").split(",")))


def run(name, spec, pods, cols, n, remote=False, steps=5, flags=0, api_ips=None, **kw):
    if ONLY and name not in ONLY:
        return
    g = GpuAgg(device=0, remote_context=remote, max_slots=len(pods.endpoints) + 16,
               max_ips=2 * len(pods.endpoints) + 16, sparse_capacity_log2=24,
               flags=flags | int(os.environ.get("ABLATE_FLAGS", "0")), **kw)
    g.reconcile(spec)
    g.load_endpoints(pods.endpoints)
    if api_ips:
        g.set_apiserver_ips(api_ips)
    dc = GpuAgg.device_columns(*cols)
    g.submit_device(dc, n)
    g.sync()
    t_settle = time.perf_counter()  # clocks settle (profiles/round5/r5k_ramp.jsonl)
    while time.perf_counter() - t_settle < float(os.environ.get("ABLATE_SETTLE_S", "0.04")):
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
    fold = st["fold_ms"] / max(1, st["kernel_launches"])
    sk = st["sketch_ms"] / max(1, st["sketch_launches"])
    print(json.dumps({"lib": os.path.basename(os.environ.get("GPUAGG_LIB", "")), "variant": name, "records": n,
                      "flags": flags | int(os.environ.get("ABLATE_FLAGS", "0")),
                      "launch_ms": ms, "fold_ms": fold, "sketch_ms": sk, "wall_ms": wall * 1e3,
                      "grec_s": n / max(ms, 1e-9) / 1e6, "hbm_frac_16B": 16 * n / (max(ms, 1e-9) * 1e-3) / 8e12}),
          flush=True)


def main():
    n = int(os.environ.get("ABLATE_N", 100_000_000))
    dev = torch.device("cuda", 0)
    pods = W.make_pods(10_000, seed=2)
    cols, _ = gen_device_records(n, pods, 2, dev, {})
    run("none", [], pods, cols, n)
    run("fwd", FWD, pods, cols, n)
    run("drop", DROP, pods, cols, n)
    run("c2", W.LOCAL_FWD_DROP, pods, cols, n)
    run("fwd-hbm-ip-table", FWD, pods, cols, n, flags=1)
    run("c2-hbm-ip-table", W.LOCAL_FWD_DROP, pods, cols, n, flags=1)
    small = W.make_pods(1_000, seed=2)
    cols_s, _ = gen_device_records(n, small, 3, dev, {})
    run("c2-1kpods", W.LOCAL_FWD_DROP, small, cols_s, n)
    del cols_s
    if not ONLY or "c4-zipf" in ONLY:  # C4: Zipf(1.2) source pods, heavy-hitter bins
        cols_z, _ = gen_device_records(n, pods, 4, dev, dict(W.CONFIGS["c4"]["gen"]))
        run("c4-zipf", W.LOCAL_FWD_DROP, pods, cols_z, n)
        del cols_z
    run("remote", W.C1_REMOTE, pods, cols, n // 10, remote=True)
    if not ONLY or any(v.startswith("c4r") for v in ONLY):  # C4 remote: Zipf 5-tuples, wide keys
        c4 = W.CONFIGS["c4-remote"]
        cols_z, _ = gen_device_records(n, pods, c4["seed"], dev, dict(c4["gen"]))
        run("c4r", W.C1_REMOTE, pods, cols_z, n, remote=True)
        run("c4r-nohot", W.C1_REMOTE, pods, cols_z, n, remote=True, flags=16)
        run("c4r-nolists", W.C1_REMOTE, pods, cols_z, n, remote=True, flags=32)
        del cols_z
    if not ONLY or "c2-lat" in ONLY:  # C2 + the latency join's filter pass (no apiserver rows)
        tcp_id = torch.zeros(n, dtype=torch.int32, device=dev)
        t_ns = torch.arange(n, dtype=torch.int64, device=dev) * 1000
        lat_spec = W.LOCAL_FWD_DROP + [{"metric_name": "node_apiserver_latency"},
                                       {"metric_name": "node_apiserver_no_response"}]
        run("c2-lat", lat_spec, pods, list(cols[:5]) + [None, tcp_id, t_ns], n,
            api_ips=[W.ip_le(10, 255, 0, 1)])
        del tcp_id, t_ns
    if not ONLY or any(v.startswith("c3") for v in ONLY):  # C3 sketch pass split by sketch
        del cols
        c3 = W.CONFIGS["c3"]
        n3 = 1 << 27
        cols3, _ = gen_device_records(n3, pods, c3["seed"], dev, dict(c3["gen"]))
        cms = dict(cms_depth=4, cms_width_log2=20)
        run("c3-none", W.LOCAL_FWD_DROP, pods, cols3, n3)
        run("c3", W.LOCAL_FWD_DROP, pods, cols3, n3, **cms, hll_precision=14)
        run("c3-cms", W.LOCAL_FWD_DROP, pods, cols3, n3, **cms)
        run("c3-cms-direct", W.LOCAL_FWD_DROP, pods, cols3, n3, flags=2, **cms)
        run("c3-hll", W.LOCAL_FWD_DROP, pods, cols3, n3, hll_precision=14)
        run("c3-hll-direct", W.LOCAL_FWD_DROP, pods, cols3, n3, flags=2, hll_precision=14)
        del cols3
        cols = None
    if not ONLY or any(v.startswith("c5") for v in ONLY):  # C5 spec split by metric
        cols = None
        c5 = W.CONFIGS["c5"]
        p5 = W.make_pods(c5["pods"], seed=c5["seed"])
        n5 = c5["records"]
        cols5, _ = gen_device_records(n5, p5, c5["seed"], dev, dict(c5["gen"]))
        spec = W.C5_SPEC
        run("c5", spec, p5, cols5, n5)
        run("c5-flags", spec[:1], p5, cols5, n5)
        run("c5-retrans", spec[1:2], p5, cols5, n5)
        run("c5-dns", spec[2:], p5, cols5, n5)
        run("c5-dense", spec[:2], p5, cols5, n5)
        run("c5-none", [], p5, cols5, n5)
        return
    if not ONLY or "raw-packet" in ONLY:
        run_raw(pods, cols, n)


def run_raw(pods, cols, n, steps=5):
    from retina_amd import _abi
    raw = W.raw_packets_torch(*cols[:5])
    g = GpuAgg(device=0, max_slots=len(pods.endpoints) + 16, max_ips=2 * len(pods.endpoints) + 16)
    g.reconcile(FWD)
    g.load_endpoints(pods.endpoints)
    g.submit_raw_device(_abi.RAW_PACKET, raw.data_ptr(), n)
    g.sync()
    g.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        g.submit_raw_device(_abi.RAW_PACKET, raw.data_ptr(), n)
    g.sync()
    wall = (time.perf_counter() - t0) / steps
    st = g.stats()
    g.close()
    dec = st["decode_ms"] / max(1, st["decode_launches"])
    agg = st["kernel_ms"] / max(1, st["kernel_launches"])
    print(json.dumps({"variant": "raw-packet", "records": n, "decode_ms": dec, "launch_ms": agg,
                      "wall_ms": wall * 1e3, "decode_grec_s": n / dec / 1e6,
                      "decode_gbs": 92 * n / (dec * 1e-3) / 1e9,
                      "decode_hbm_frac": 92 * n / (dec * 1e-3) / 8e12}), flush=True)


if __name__ == "__main__":
    main()
