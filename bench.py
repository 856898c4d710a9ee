"""Benchmark: flow records/s aggregated on MI355X (BASELINE.json metric).

Workload (config C2): a 100M-record batch of synthetic decoded flows,
10k pods, local context, per-pod forward count/bytes + drop-reason histogram
(forward_count, forward_bytes, drop_count, drop_bytes with sourceLabels
[namespace, podname]).  One step = one aggregation pass over the whole batch, with
the records already resident in HBM.  Weak scaling: every rank aggregates its own
100M-record shard; the counters are merged once per timed region with an RCCL
all-reduce (the per-scrape-epoch merge).

    python bench.py [--gpus N --steps K --warmup W --config c2 --records R]

Other BASELINE.json configs (parity-test cases; bench lines under profiles/):
  --config c3   2^27 records per GPU (2^30 on 8 GPUs), C2 metrics + count-min
                (d=4, w=2^20) over the 5-tuple + HLL p=14 of distinct dst per source pod;
                counters, count-min (sum) and HLL registers (max) merged per timed region
  --config c4   C2 with Zipf(1.2) source pods (atomic contention on heavy hitters)
  --config c5   10M records, 100k pods: tcpflags + retransmits + DNS request/response
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
# Algorithmic bytes per record: the columns the enabled metrics read.
# C5's metrics (tcpflags, retransmits, DNS) count records only: src, dst, meta, dns_id.
BYTES_PER_RECORD = {"c1": 16, "c2": 16, "c3": 20, "c4": 16, "c4-src": 16, "c4-remote": 16, "c5": 16}
REMOTE_CONFIGS = {"c4-remote"}  # remote context: source and destination label tuples
# the sketch pass reads src, dst, ports, meta (proto)
SKETCH_BYTES_PER_RECORD = 16


def bench_spec(name: str):
    """(metric spec, sketch kwargs, workload text) of a BASELINE.json config."""
    from retina_amd import workloads as W
    c2txt = "local context, per-pod forward count/bytes + drop-reason histogram [namespace, podname]"
    if name == "c1":
        return W.C1_LOCAL, {}, "C1 spec: local context [ip, namespace, podname, workload], forward + drop"
    if name == "c3":
        return W.LOCAL_FWD_DROP, dict(cms_depth=4, cms_width_log2=20, hll_precision=14), (
            "C3: " + c2txt + " + count-min d=4 w=2^20 over the 5-tuple + HLL p=14 distinct dst per source pod")
    if name == "c4":
        return W.LOCAL_FWD_DROP, {}, "C4: Zipf(1.2) 5-tuple ranks over 10^7 flows, " + c2txt
    if name == "c4-remote":
        return W.C1_REMOTE, {}, ("C4 remote context: Zipf(1.2) 5-tuple ranks over 10^7 flows, forward + drop "
                                 "[ip, namespace, podname, workload] on both sides (sparse group-by keys)")
    if name == "c4-src":
        return W.LOCAL_FWD_DROP, {}, "C4 (round-1 form): Zipf(1.2) source pods, " + c2txt
    if name == "c5":
        return W.C5_SPEC, {}, "C5: tcpflags + tcp retransmission + DNS request/response, local context [namespace, podname]"
    return W.LOCAL_FWD_DROP, {}, "C2: " + c2txt


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gen_device_records(n: int, pods, seed: int, device, gen_kw, chunk: int = 8_000_000, cache_key: str = ""):
    """Generates the workload on the host in chunks and keeps it resident in HBM.  With
    BENCH_CACHE=<dir> (the profiling sessions' repeated runs) the generated columns and the
    last chunk's DNS payloads are kept as .npy / JSON files and reused by the next run."""
    import torch
    from retina_amd import workloads as W
    cache = os.environ.get("BENCH_CACHE", "")
    if cache and cache_key:
        base = os.path.join(cache, "%s_%d_%d" % (cache_key, n, seed))
        if os.path.exists(base + ".json"):
            dns = [W.DnsPayload(**d) for d in json.load(open(base + ".json"))]
            cols = [torch.from_numpy(np.load(base + "_%d.npy" % k)).to(device) for k in range(6)]
            return cols, W.Records(*[None] * 6, dns)
    cols = [torch.empty(n, dtype=torch.int32, device=device) for _ in range(6)]
    start, k = 0, 0
    while start < n:
        m = min(chunk, n - start)
        r = W.gen_records(m, pods, seed * 1000 + k, **gen_kw)
        for t, a in zip(cols, (r.src_ip, r.dst_ip, r.bytes, r.meta, r.ports, r.dns_id)):
            t[start:start + m].copy_(torch.from_numpy(a.view(np.int32)))
        start += m
        k += 1
    if cache and cache_key:
        os.makedirs(cache, exist_ok=True)
        for k, t in enumerate(cols):
            np.save(base + "_%d.npy" % k, t.cpu().numpy())
        with open(base + ".json", "w") as f:  # written last: marks the entry complete
            json.dump([vars(p) for p in r.dns], f)
    return cols, r


def _cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    # the GPU box grants a 16-CPU share of a larger machine (OMP_NUM_THREADS=16 there)
    share = int(os.environ.get("OMP_NUM_THREADS", avail) or avail)
    return model, os.cpu_count() or 1, max(1, min(avail, share))


def cpu_baseline(cfg_name: str, pods, spec, seed: int, gen_kw, go_sample: int, tuned_sample: int,
                 runs: int = 5, remote: bool = False):
    """The C port of the reference path (oracle/ref_cpu.c) timed on this host, in the two
    modes of SURVEY.md 8d / BASELINE.md, 1 warm-up + `runs` timed runs each, median:
      go-shaped: dotted-string IPs, string-keyed cache and label maps, enrich + every
                 ProcessFlow per flow on one thread (enricher.go:69-98,
                 metrics_module.go:276-317);
      tuned:     integer keys, every granted core, per-thread tables merged at the end.
    `value` is the tuned median (the stronger CPU baseline)."""
    from oracle.ref_cpu import RefCPU
    from retina_amd import workloads as W
    model, ncpu, threads = _cpu_info()
    recs = W.gen_records(tuned_sample, pods, seed, **gen_kw)
    go = W.Records(*(getattr(recs, k)[:go_sample] for k in ("src_ip", "dst_ip", "bytes", "meta",
                                                              "ports", "dns_id")), recs.dns)

    def timed(fn, n):
        rates = []
        for i in range(runs + 1):
            r = RefCPU(spec, pods.endpoints, remote, recs.dns)
            dt = fn(r)
            r.close()
            if i:  # run 0 is the warm-up
                rates.append(n / dt)
        return float(np.median(rates)), rates

    go_med, go_all = timed(lambda r: r.process(go), go_sample)
    tu_med, tu_all = timed(lambda r: r.process_tuned(recs, threads), tuned_sample)
    return {"value": tu_med, "unit": "records/s", "cores": threads, "kind": "port",
            "sample": "config %s through oracle/ref_cpu.c (C port of enricher.go + metrics module); "
                      "tuned: %d records on %d threads; go-shaped: %d records on 1 thread; "
                      "1 warm-up + %d timed runs each, median" % (cfg_name, tuned_sample, threads,
                                                                 go_sample, runs),
            "cpu_model": model, "nproc": ncpu,
            "modes": {"tuned": {"value": tu_med, "threads": threads, "records": tuned_sample,
                                "runs": tu_all},
                      "go_shaped": {"value": go_med, "threads": 1, "records": go_sample,
                                    "runs": go_all}}}


def pmc_traffic(cfg_name: str, kernel: str, build_id: str):
    """HBM bytes per launch from profiles/pmc_<config>.json, only if that file profiles
    the kernel that ran (its `kernel` list holds rocprofv3 names containing `kernel`) AND
    was collected from the same library build (its `build_id` equals gpuagg_build_id(),
    a hash of retina_amd/csrc/*): counters of older code are never reported."""
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % cfg_name)
    if not os.path.exists(path):
        return None, "no %s" % os.path.relpath(path, ROOT)
    try:
        pmc = json.load(open(path))
    except ValueError:
        return None, "unreadable %s" % os.path.relpath(path, ROOT)
    names = pmc.get("kernel", [])
    # a composite "a+b+c" (the sketch pass) needs every part profiled
    parts = [p for p in (kernel or "").split("+") if p]
    if not parts or not all(any(p in k for k in names) for p in parts):
        return None, "%s profiles %s, not %s: refused" % (os.path.relpath(path, ROOT), names, kernel)
    if pmc.get("build_id") != build_id:
        return None, "%s is from build %s, this library is %s: refused" % (
            os.path.relpath(path, ROOT), pmc.get("build_id"), build_id)
    return pmc.get("hbm_bytes_per_launch_corrected"), os.path.relpath(path, ROOT)


# Secondary ceilings of MI355X measured by scripts/microbench_bounds.hip on the box
# (profiles/round6/r6b_bounds.jsonl), for the kernels that are not HBM-streaming-bound:
SECONDARY_PEAKS = {
    # random u32 adds into a 64 KiB LDS array, one 1024-thread workgroup per CU (ds_add_u32)
    "lds_atomic": {"peak": 4.46e12, "unit": "lane atomics/s"},
    # random 4-byte loads from an L2-resident 1 MiB table (one L2 request each)
    "l2_gather": {"peak": 2.73e11, "unit": "L2 requests/s"},
    # the LDS array's cycles: SQ_LDS_IDX_ACTIVE over the CUs' cycles of the launch
    "lds_array": {"peak": 1.0, "unit": "busy fraction"},
}
N_CU, N_XCD = 256, 8


def secondary_bounds(pmc_path, kernel_ms: float):
    """The dominant kernel's use of its non-HBM resources against SECONDARY_PEAKS, from the
    same PMC file (and build) as `traffic`: LDS atomics (SQ_INSTS_LDS_ATOMIC x 64 lanes),
    L2 requests (TCC_HIT + TCC_MISS) and LDS-array busy cycles (SQ_LDS_IDX_ACTIVE over
    CUs x GRBM_GUI_ACTIVE / XCDs), per launch over the kernel's HIP-event time.  `bound` is
    the resource with the largest fraction."""
    try:
        c = json.load(open(os.path.join(ROOT, pmc_path)))["counters_avg_per_dispatch"]
    except (OSError, ValueError, KeyError, TypeError):
        return None
    s = kernel_ms * 1e-3
    out = {}
    if "SQ_INSTS_LDS_ATOMIC" in c:
        a = c["SQ_INSTS_LDS_ATOMIC"] * 64 / s
        out["lds_atomic"] = {"achieved": a, "frac": a / SECONDARY_PEAKS["lds_atomic"]["peak"]}
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        a = (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) / s
        out["l2_gather"] = {"achieved": a, "frac": a / SECONDARY_PEAKS["l2_gather"]["peak"]}
    if c.get("SQ_LDS_IDX_ACTIVE") and c.get("GRBM_GUI_ACTIVE"):
        a = c["SQ_LDS_IDX_ACTIVE"] / (N_CU * c["GRBM_GUI_ACTIVE"] / N_XCD)
        out["lds_array"] = {"achieved": a, "frac": a}
    for k, v in out.items():
        v.update(peak=SECONDARY_PEAKS[k]["peak"], unit=SECONDARY_PEAKS[k]["unit"])
    if out:
        out["bound"] = max((k for k in out), key=lambda k: out[k]["frac"])
        out["source"] = "%s + profiles/round6/r6b_bounds.jsonl" % pmc_path
    return out


# The Go plugin's batch geometry (go/pkg/gpuagg/gpuagg_linux.go): the packetparser feed's
# stagings hold packetCapacity = 2^22 raw samples (the traffic path; submitted when full or
# every flushInterval = 100 ms), decoded records and drops batchCapacity = 2^20 (round 6;
# every feed took 2^22 in round 5, 2^20 before).
GO_BATCH = 1 << 22
RECORD_BATCH = 1 << 20


def host_fed_rate(g, cols, n_total: int, steps: int, batch: int = RECORD_BATCH):
    """Host-fed throughput at the Go plugin's decoded-record batch size: two pinned batches (pre-filled
    from the workload) submitted alternately through gpuagg_submit, the H2D copy of one
    overlapping the other's aggregation."""
    import torch
    n = min(batch, n_total)
    hbs = [g.alloc_batch(n), g.alloc_batch(n)]
    for k, hb in enumerate(hbs):
        lo = (k * n) % max(1, n_total - n + 1)
        for name, t in zip(("src_ip", "dst_ip", "bytes", "meta", "ports", "dns_id"), cols):
            getattr(hb, name)[:n] = t[lo:lo + n].cpu().numpy().view(np.uint32)
    g.submit(hbs[0], n)
    g.sync()
    torch.cuda.synchronize()
    reps = max(4, steps * 4)
    t0 = time.perf_counter()
    for k in range(reps):
        g.submit(hbs[k & 1], n)
    g.sync()
    dt = time.perf_counter() - t0
    return {"value": reps * n / dt, "unit": "records/s", "batch_records": n, "batches": reps,
            "note": "pinned host batches through gpuagg_submit (PCIe H2D included; not `value`)"}


def host_fed_raw_rate(g, pods, spec, seed: int, batches: int = 12, batch: int = GO_BATCH):
    """The Go plugin's raw path (gpuagg_linux.go Start -> submitRaw): raw 72-byte
    packetparser samples (conntrack.c:34-49) handed to the library feed in 2^16-sample
    pieces (rawPiece) -- gpuagg_raw_feed_put: the feed's host threads shard by the 5-tuple
    and write into one of the device's two pinned GO_BATCH-record stagings; a full staging's
    H2D DMA starts without a wait while the other fills -- then a flush and sync.
    `value`: the feed's defaults -- samples copied as they are (72 B per record over PCIe)
    and decoded on the GPU (GPUAGG_FEED_RAW_DMA), 4 feed threads; `modes` times both modes
    (GPUAGG_FEED_HOST_DECODE: decoded on the feed's threads, only the columns the metrics
    read cross PCIe) at 1-16 feed threads, and
    `shard8`: the same feed over 8 contexts of this one GPU (the 8-device node's shard +
    scatter path; the 8 stagings share this GPU and its PCIe link).  `shard_rate_8_devices`
    times gpuagg_shard_raw alone (its host threads)."""
    from retina_amd import GpuAgg, RawFeed, _abi
    from retina_amd import workloads as W
    raw = W.gen_raw_packets(batch, pods, seed=seed)  # one Go batch of samples, resubmitted
    piece = 1 << 16

    def run(engines, mode, threads, nb, cap=batch):
        feed = RawFeed(engines, _abi.RAW_PACKET, capacity=cap, threads=threads, mode=mode)
        try:
            for a in range(0, batch, piece):  # warm-up: stagings, device buffers, pool threads
                feed.put(raw[a * 72:(a + piece) * 72])
            feed.flush()
            for e in set(engines):
                e.sync()
            t0 = time.perf_counter()
            for _ in range(nb):
                for a in range(0, batch, piece):
                    feed.put(raw[a * 72:(a + piece) * 72])
            feed.flush()
            for e in set(engines):
                e.sync()
            return nb * batch / (time.perf_counter() - t0)
        finally:
            feed.close()

    modes = {}
    for name, mode in (("host_decode", _abi.FEED_HOST_DECODE), ("raw_dma", _abi.FEED_RAW_DMA)):
        modes[name] = {str(t): run([g], mode, t, batches) for t in (1, 2, 4, 8, 16)}
    best = max(((m, t) for m in modes for t in modes[m]), key=lambda mt: modes[mt[0]][mt[1]])
    # 8 contexts on this GPU, the plan of `g` (the shard + scatter path of an 8-GPU node)
    extra = [GpuAgg(device=g.device, remote_context=False, max_slots=len(pods.endpoints) + 16,
                    max_ips=2 * len(pods.endpoints) + 16) for _ in range(7)]
    try:
        for e in extra:
            e.reconcile(spec)
            e.load_endpoints(pods.endpoints)
        # (stagings of batch / 4 records here: 8 contexts x 2 stagings of 72-byte samples)
        shard8 = {name: {str(t): run([g] + extra, mode, t, batches // 2, batch // 4) for t in (4, 8, 16)}
                  for name, mode in (("host_decode", _abi.FEED_HOST_DECODE), ("raw_dma", _abi.FEED_RAW_DMA))}
        # the host side alone (FEED_DRY_RUN: stagings counted, never copied or aggregated):
        # what the node's CPU can shard + scatter (+ decode) into 8 devices' pinned stagings
        # when every device has its own PCIe link
        shard8_host = {name: {str(t): run([g] + extra, mode | _abi.FEED_DRY_RUN, t, batches // 2, batch // 4)
                              for t in (1, 4, 8, 16)}
                       for name, mode in (("host_decode", _abi.FEED_HOST_DECODE), ("raw_dma", _abi.FEED_RAW_DMA))}
    finally:
        for e in extra:
            e.close()
    shards = np.zeros(batch, np.uint32)
    t1 = time.perf_counter()
    for _ in range(8):
        rc = g.lib.gpuagg_shard_raw(_abi.RAW_PACKET, raw.ctypes.data_as(C.c_void_p), batch, 8,
                                    shards.ctypes.data_as(_abi.u32p))
        if rc != 0:
            raise RuntimeError("gpuagg_shard_raw: %d" % rc)
    shard_rate = 8 * batch / (time.perf_counter() - t1)
    return {"value": modes["raw_dma"]["4"], "unit": "records/s", "batch_records": batch, "batches": batches,
            "piece_records": piece, "record_bytes": 72, "feed_threads": 4, "feed_mode": "raw_dma", "modes": modes,
            "best": {"mode": best[0], "threads": int(best[1]), "value": modes[best[0]][best[1]]},
            "shard8": shard8, "shard8_host_only": shard8_host, "shard_rate_8_devices": shard_rate,
            "note": "raw packetparser samples through gpuagg_raw_feed_put in 2^16-sample pieces, 2 pinned 2^22-record "
                    "stagings per context, async H2D -- the Go plugin's real raw path; PCIe included, not `value`. "
                    "value = the feed's defaults (raw_dma, 4 threads); modes = records/s by mode and feed threads; shard8 = "
                    "one feed over 8 contexts of this GPU; shard8_host_only = the same with the DMA and aggregation out of the "
                    "loop (GPUAGG_FEED_DRY_RUN: the host's shard + scatter + decode ceiling for an 8-GPU node); "
                    "shard_rate_8_devices = gpuagg_shard_raw (threaded) samples/s"}


def production_geometry(g, cols, n_total: int, bpr: int, full_kernel_ms: float, launches: int = 100,
                        batch: int = GO_BATCH):
    """Device-resident launches of the Go plugin's batch size (GO_BATCH records each): the
    per-launch fixed cost next to the headline's one big launch.  fixed_ms = the kernel's
    time per launch minus the time the same records take at the full-size launch's rate
    (LDS image fill, bin zeroing and flush, staged copies, spill folds do not shrink with
    the batch)."""
    from retina_amd import GpuAgg
    n = min(batch, n_total)
    sub = GpuAgg.device_columns(*[t[:n] for t in cols])
    g.submit_device(sub, n)
    g.sync()
    g.set_timing(False)
    # wall rate untimed (HIP events between launches would add gaps the plugin never has),
    # then the same launches timed for the kernel split
    t0 = time.perf_counter()
    for _ in range(launches):
        g.submit_device(sub, n)
    g.sync()
    wall = (time.perf_counter() - t0) / launches
    g.set_timing(True)
    for _ in range(launches):
        g.submit_device(sub, n)
    g.sync()
    st = g.stats()
    g.set_timing(False)
    k = st["kernel_launches"] or 1
    kms = st["kernel_ms"] / k
    other = (st["fold_ms"] + st["sketch_ms"]) / k  # folds and the sketch pass, per aggregation launch
    at_full_rate = full_kernel_ms * n / n_total
    return {"batch_records": n, "launches": launches, "records_per_s": n / wall, "ms_per_launch": wall * 1e3,
            "kernel_ms": kms, "other_kernels_ms": other,
            "kernel_frac": bpr * n / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "fixed_ms": kms - at_full_rate,
            "note": "device-resident %d-record launches (Go batchCapacity), wall rate untimed; kernel_ms / "
                    "other_kernels_ms from a HIP-event-timed repeat; fixed_ms = kernel ms per launch - the same "
                    "records at the full-size launch's rate" % n}


# Prometheus' default scrape interval: the engine's snapshot + text rendering is a host cost
# paid once per scrape epoch (prometheusexporter.go:19,29-31 serve the registry per scrape).
SCRAPE_EPOCH_S = 15.0


def scrape_cost(g, reps: int = 3):
    """Host-side cost of one scrape on the state the timed region left: gpuagg_snapshot
    (device sync, table compaction and D2H, label rendering of every series) and
    gpuagg_result_text (client_golang's text exposition, rendered once and handed out
    without a copy; the copying gpuagg_result_render_text is timed beside it), median of
    `reps` after a first, cold scrape
    (whose snapshot also builds the canonical label tables, as a scrape does after pod churn
    or new DNS payloads).  The walk a Go publish does over the result is not included."""
    snap, rend, copy, nser, nbytes = [], [], [], 0, 0
    out = None
    for _ in range(reps + 1):
        r = C.c_void_p()
        t0 = time.perf_counter()
        rc = g.lib.gpuagg_snapshot(g.h, C.byref(r))
        t1 = time.perf_counter()
        if rc != 0:
            raise RuntimeError("gpuagg_snapshot: %d" % rc)
        try:
            nser = int(g.lib.gpuagg_result_count(r))
            ln = C.c_size_t()
            ptr = C.c_void_p()
            t2 = time.perf_counter()
            rc = g.lib.gpuagg_result_text(r, C.byref(ptr), C.byref(ln))  # renders; no copy
            t3 = time.perf_counter()
            if out is None or out.size < ln.value + 1:
                out = np.empty(ln.value + 1, np.uint8)
            t4 = time.perf_counter()
            # the copying form (gpuagg_result_render_text into a caller buffer), for reference
            rc = rc or g.lib.gpuagg_result_render_text(r, out.ctypes.data_as(C.c_char_p), out.size, C.byref(ln))
            t5 = time.perf_counter()
            if rc != 0:
                raise RuntimeError("gpuagg_result_render_text: %d" % rc)
            nbytes = int(ln.value)
        finally:
            g.lib.gpuagg_result_free(r)
        snap.append((t1 - t0) * 1e3)
        rend.append((t3 - t2) * 1e3)
        copy.append((t5 - t4) * 1e3)
    sm, rm, cm = (float(np.median(x[1:])) for x in (snap, rend, copy))
    return {"series": nser, "text_bytes": nbytes, "snapshot_ms": sm, "render_ms": rm, "copy_ms": cm,
            "cold_snapshot_ms": snap[0], "cold_render_ms": rend[0],
            "epoch_frac": (sm + rm) / (SCRAPE_EPOCH_S * 1e3),
            "cold_epoch_frac": (snap[0] + rend[0]) / (SCRAPE_EPOCH_S * 1e3), "epoch_s": SCRAPE_EPOCH_S,
            "note": "gpuagg_snapshot + gpuagg_result_text (the exposition rendered, handed out without a copy) on "
                    "the timed region's state: median of %d warm scrapes, and the first (cold) one; copy_ms is the "
                    "extra cost of the copying form gpuagg_result_render_text (not in epoch_frac); host cost per "
                    "scrape epoch, outside `value`" % reps}


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: run N rank processes of this
    script under torch.distributed.run (one per GPU, 127.0.0.1 rendezvous) as a CHILD and
    return its exit code.  Called before anything in this process touches the GPU (no exec
    from a process with a HIP context); every rank then binds its device before joining the
    process group (rank_device / main)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    return subprocess.call(cmd + list(argv), env=env)


def rank_device(local_rank: int, local_world: int, backend: str, ndev: int) -> int:
    """The GPU of a rank: one per rank (RCCL needs distinct devices).  Under gloo, ranks may
    share devices round-robin (the one-GPU rehearsal of the multi-rank path)."""
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible (use --cpu-backend for the host engine)")
    if local_world > ndev:
        if backend == "nccl":
            raise SystemExit("bench.py: %d ranks on %d visible GPUs: RCCL needs one GPU per rank "
                             "(--backend gloo shares devices)" % (local_world, ndev))
        return local_rank % ndev
    return local_rank


def host_columns(arrs):
    """_abi.Columns over host numpy arrays (the CPU backend's "device" memory)."""
    from retina_amd import _abi
    return _abi.Columns(*[a.ctypes.data_as(_abi.u32p) for a in arrs], None, None)


def gen_host_records(n: int, pods, seed: int, gen_kw, chunk: int = 8_000_000):
    """gen_device_records for the CPU backend: the same columns, kept in host memory."""
    from retina_amd import workloads as W
    cols = [np.empty(n, np.uint32) for _ in range(6)]
    start, k, r = 0, 0, None
    while start < n:
        m = min(chunk, n - start)
        r = W.gen_records(m, pods, seed * 1000 + k, **gen_kw)
        for t, a in zip(cols, (r.src_ip, r.dst_ip, r.bytes, r.meta, r.ports, r.dns_id)):
            t[start:start + m] = a
        start += m
        k += 1
    return cols, r


def merge_check(args, cfg, spec, sketch, remote, n, world, g, gen, cols_of, pods, gen_kw, chunk, capacity):
    """--check-merge: rank 0's merged state after the timed region against ONE engine fed
    every rank's batch `steps` times (the engine was reset after the warm-up, so the merged
    state holds exactly the timed steps of every rank).  Counters and count-min are sums and
    HLL registers a max, so the two must be equal bit for bit."""
    from retina_amd import GpuAgg
    ref = GpuAgg(device=g.device, remote_context=remote, max_slots=cfg["pods"] + 16,
                 max_ips=2 * cfg["pods"] + 16, sparse_capacity_log2=capacity, flags=g.cfg.flags, **sketch)
    try:
        ref.reconcile(spec)
        ref.load_endpoints(pods.endpoints)
        for r in range(world):
            cols, _ = gen(n, pods, cfg["seed"] + 7919 * r, gen_kw, chunk)
            dc = cols_of(cols)
            for _ in range(args.steps):
                ref.submit_device(dc, n)
            ref.sync()
        want, got = ref.snapshot(), g.snapshot()
        out = {"series": len(got), "series_equal": got == want, "records_each_rank": n, "ranks": world}
        if sketch:
            out["cms_equal"] = bool(np.array_equal(g.cms_array(), ref.cms_array()))
            out["hll_equal"] = bool(np.array_equal(g.hll_array(), ref.hll_array()))
        out["equal"] = all(v for k, v in out.items() if k.endswith("_equal"))
        return out
    finally:
        ref.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=0,
                    help="GPUs (ranks) of this node; default: WORLD_SIZE, or 1.  Without a launcher, "
                         "N > 1 starts N ranks under torch.distributed.run")
    ap.add_argument("--backend", default=os.environ.get("GPUAGG_BENCH_BACKEND", "nccl"),
                    choices=("nccl", "gloo"),
                    help="collective backend of the per-epoch merge: nccl = RCCL over xGMI; gloo stages "
                         "through host memory and lets ranks share one GPU")
    ap.add_argument("--cpu-backend", action="store_true",
                    help="run the engine's CPU backend (GPUAGG_FLAG_CPU_BACKEND, host memory) instead of "
                         "a GPU: rehearses the multi-rank path on a machine without one (not a bench line)")
    ap.add_argument("--check-merge", action="store_true",
                    help="reset the engines after the warm-up, and after the timed region check rank 0's "
                         "merged state against one engine fed every rank's batch")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--records", type=int, default=0, help="records per GPU (default: config size)")
    ap.add_argument("--cpu-sample", type=int, default=16_000_000,
                    help="records in the tuned CPU baseline sample (go-shaped: 1/8 of it)")
    ap.add_argument("--settle-ms", type=float, default=40.0,
                    help="untimed passes of the step for this long before the warm-up steps (clock settle)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-fed", action="store_true")
    ap.add_argument("--no-scrape", action="store_true", help="skip the snapshot / render timing")
    ap.add_argument("--production-only", action="store_true",
                    help="diagnostic: only the production-geometry launches (for rocprof), no bench line")
    ap.add_argument("--no-production", action="store_true",
                    help="skip the Go-batch-size (1M-record) device-resident launches")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # nothing has touched the GPU yet (torch is not even imported): start the ranks
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.gpus and args.gpus != world:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.cpu_backend and args.backend != "gloo":
        raise SystemExit("bench.py: --cpu-backend merges over gloo (pass --backend gloo)")
    if args.check_merge and args.config == "c5":
        # DNS ids index each rank's own generated payload dictionary; the merge of DNS keys
        # needs one dictionary interned alike on every rank (as the Go plugin does per context)
        raise SystemExit("bench.py: --check-merge does not cover c5 (per-rank DNS dictionaries)")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))

    import torch
    import torch.distributed as dist
    from retina_amd import GpuAgg, _abi
    from retina_amd import workloads as W
    from retina_amd.dist import merge_engine

    cpu = args.cpu_backend
    if cpu:
        dev_index, device = 0, torch.device("cpu")
    else:
        # bind this rank's GPU BEFORE the process group exists (RCCL communicators are made
        # on the current device)
        dev_index = rank_device(local_rank, local_world, args.backend, torch.cuda.device_count())
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    if world > 1:
        dist.init_process_group(args.backend)
        if dist.get_world_size() != world:
            raise SystemExit("bench.py: process group has %d ranks, WORLD_SIZE %d" % (dist.get_world_size(), world))
    cuda_sync = (lambda: None) if cpu else torch.cuda.synchronize

    cfg = W.CONFIGS[args.config]
    n = args.records or cfg["records"]
    if args.config == "c3" and not args.records:
        n = cfg["records"] // 8  # 2^30 records over the 8 GPUs of a node; weak scaling per GPU
    gen_kw = dict(cfg["gen"])
    spec, sketch, workload = bench_spec(args.config)
    bpr = BYTES_PER_RECORD[args.config]
    pods = W.make_pods(cfg["pods"], seed=cfg["seed"])
    t0 = time.time()
    # DNS ids index one generated dictionary: C5 is generated as a single chunk
    chunk = n if args.config == "c5" else 8_000_000
    if cpu:
        def gen(nn, pp, seed, kw, ch):
            return gen_host_records(nn, pp, seed, kw, chunk=ch)
        cols_of = host_columns
    else:
        def gen(nn, pp, seed, kw, ch):
            return gen_device_records(nn, pp, seed, device, kw, chunk=ch)
        cols_of = lambda c: GpuAgg.device_columns(*c)  # noqa: E731
    if cpu or world > 1:
        cols, last = gen(n, pods, cfg["seed"] + 7919 * rank, gen_kw, chunk)
    else:
        cols, last = gen_device_records(n, pods, cfg["seed"], device, gen_kw, chunk=chunk, cache_key=args.config)
    cuda_sync()
    log("rank %d: %d records resident in %s (%.1f s)" % (rank, n, "host memory" if cpu else "HBM of cuda:%d" % dev_index,
                                                        time.time() - t0))

    # C5's DNS series are sparse keys (one per query payload and side): a 2^24-slot table
    remote = args.config in REMOTE_CONFIGS
    capacity = {"c1": 21, "c5": 23, "c4-remote": 24}.get(args.config, 16)
    g = GpuAgg(device=dev_index, remote_context=remote, max_slots=cfg["pods"] + 16,
               max_ips=2 * cfg["pods"] + 16, sparse_capacity_log2=capacity,
               flags=(_abi.FLAG_CPU_BACKEND if cpu else 0) | int(os.environ.get("GPUAGG_BENCH_FLAGS", "0"), 0),
               **sketch)  # (GPUAGG_BENCH_FLAGS: diagnostic gpuagg_config.flags for A/B runs)
    g.reconcile(spec)
    g.load_endpoints(pods.endpoints)
    for p in last.dns:
        g.dns_intern(p.rcode, p.qtypes, p.query, p.ips, p.num_answers)
    dcols = cols_of(cols)

    if args.production_only:  # diagnostic (rocprof of the GO_BATCH-record launches)
        print(json.dumps({"production": production_geometry(g, cols, n, bpr, 0.0)}), flush=True)
        g.close()
        return

    # settle: untimed passes of the same step until the GPU's clocks reach the steady
    # state an always-on agent runs at.  After idle the tier-1 kernel's time rises for
    # ~10 launches and settles after ~25 (0.409 -> 0.425 -> 0.404 ms at C2, the same after
    # 2 s idle: profiles/round5/r5k_ramp.jsonl), so the driver's 5 warm-up steps left the
    # timed region in the hump.  Reported as `settle`; the timed region is unchanged.
    # Launches go back to back in groups of 8 (a sync after each one left the GPU idle for a
    # host round trip per launch, which at C1's 56 us launches showed in rocprof's averages).
    settle_n, t_settle = 0, time.perf_counter()
    while args.settle_ms > 0 and (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        for _ in range(8):
            g.submit_device(dcols, n)
        g.sync()
        settle_n += 8
    settle_s = time.perf_counter() - t_settle
    for _ in range(args.warmup):
        g.submit_device(dcols, n)
    g.sync()
    if world > 1:  # an untimed merge first: RCCL communicators and merge buffers exist before the clock
        merge_engine(g)
    if args.check_merge:  # the state then holds exactly the timed steps
        g.reset()

    # ---- timed region --------------------------------------------------------------
    if world > 1:
        dist.barrier()
    cuda_sync()
    g.set_timing(False)
    g.set_timing(True)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        g.submit_device(dcols, n)
    g.sync()
    t_merge = time.perf_counter()
    if world > 1:  # per-epoch merge over RCCL/xGMI: dense + count-min sum, HLL max, sparse table
        merge_engine(g)
    cuda_sync()
    if world > 1:
        dist.barrier()
    t_end = time.perf_counter()
    elapsed, merge_s = t_end - t_start, t_end - t_merge
    stats = g.stats()
    kernel = g.kernel_name()
    sketch_kernels = g.sketch_kernel_name()
    g.set_timing(False)
    if stats["sparse_dropped"]:
        raise RuntimeError("group-by table overflowed (%d updates lost)" % stats["sparse_dropped"])
    # max over ranks (a gloo group reduces host tensors)
    t = torch.tensor([elapsed, merge_s], dtype=torch.float64,
                     device=device if (world > 1 and args.backend == "nccl") else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, merge_s = (float(x) for x in t.tolist())

    # roofline of the dominant kernel: the aggregation kernel, or (C3) the sketch pass
    agg_ms = stats["kernel_ms"] / max(1, stats["kernel_launches"])
    fold_ms = stats["fold_ms"] / max(1, stats["kernel_launches"])
    sk_ms = stats["sketch_ms"] / max(1, stats["sketch_launches"]) if stats["sketch_launches"] else 0.0
    if sk_ms > agg_ms:
        dom, dom_ms, dom_bpr = sketch_kernels, sk_ms, SKETCH_BYTES_PER_RECORD
        other_ms = agg_ms + fold_ms
    else:
        dom, dom_ms, dom_bpr = kernel, agg_ms, bpr
        other_ms = fold_ms + sk_ms
    achieved = dom_bpr * n / (dom_ms * 1e-3) / 1e9
    build_id = g.lib.gpuagg_build_id().decode()
    traffic, traffic_src = pmc_traffic(args.config, dom, build_id)

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
            "workload": "%s; %d-record batch per GPU, %d pods" % (workload, n, cfg["pods"]),
            "records_per_gpu": n,
            "pods": cfg["pods"],
            "metrics": [s["metric_name"] for s in spec],
            "parallelism": "dp%d (records sharded, state merged once per timed region)" % world,
            "backend": "cpu engine (GPUAGG_FLAG_CPU_BACKEND; rehearsal, not a GPU measurement)" if cpu
            else ("gfx950; merge over %s" % ("RCCL" if args.backend == "nccl" else "gloo") if world > 1
                  else "gfx950"),
        },
        "merge_ms": merge_s * 1e3 if world > 1 else None,
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": dom,
            "kernel_ms": dom_ms,
            "other_kernels_ms": other_ms,
            "bytes_per_record": dom_bpr,
            "step_bytes_per_record": bpr,
            "secondary": secondary_bounds(traffic_src, dom_ms) if traffic is not None else None,
        },
        "build_id": build_id,
        "settle": {"launches": settle_n, "s": settle_s,
                   "note": "untimed passes of the step before the warm-up steps, so the timed region runs at "
                           "steady-state clocks (profiles/round5/r5k_ramp.jsonl)"},
    }
    if cpu:  # the host engine: no kernel, no HBM roofline
        result["roofline"] = None
    if args.check_merge and rank == 0:
        result["merge_check"] = merge_check(args, cfg, spec, sketch, remote, n, world, g, gen, cols_of, pods,
                                            gen_kw, chunk, capacity)
    if rank == 0 and not args.no_scrape:
        result["scrape"] = scrape_cost(g)
    if rank == 0 and world == 1 and not cpu and not args.no_production and n > GO_BATCH:
        result["production"] = production_geometry(g, cols, n, bpr, stats["kernel_ms"] / max(1, stats["kernel_launches"]))
    if rank == 0 and world == 1 and not cpu and not args.no_host_fed:
        result["host_fed"] = host_fed_rate(g, cols, n, args.steps)
        result["host_fed_raw"] = host_fed_raw_rate(g, pods, spec, cfg["seed"] + 17)
    if rank == 0 and world == 1 and not cpu and not args.no_cpu_baseline:
        go_s, tu_s = (400_000, 4_000_000) if args.config == "c5" else (args.cpu_sample // 8, args.cpu_sample)
        result["cpu_baseline"] = cpu_baseline(args.config, pods, spec, cfg["seed"], gen_kw, go_s, tu_s,
                                              remote=remote)
        if sketch:
            result["cpu_baseline"]["sample"] += " (metrics only: the sketches have no reference CPU path)"
    g.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
