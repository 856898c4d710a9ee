"""Rows of BASELINE.md's results table from bench lines (one JSON per config).

    python scripts/baseline_table.py profiles/round3/f3b_bench_c1.json [...]
"""

import json
import sys

LABEL = {
    "c1": "C1 (1M, local ip/ns/pod/workload keys)",
    "c2": "C2 (100M, 10k pods, fwd + drop)",
    "c3": "C3 (2^27 per GPU, + CMS d=4 w=2^20 + HLL p=14)",
    "c4": "C4 (Zipf 1.2 5-tuples)",
    "c4-remote": "C4 remote context (sparse keys)",
    "c5": "C5 (10M, 100k pods, tcpflags + retrans + DNS)",
}


def pow2(n: int) -> str:
    return "2^%d" % (n.bit_length() - 1) if n and not n & (n - 1) else str(n)


def rows(path):
    d = json.load(open(path))
    cfg = path.rsplit("_bench_", 1)[-1].replace(".json", "")
    r = d["roofline"]
    cpu = d.get("cpu_baseline") or {}
    out = []
    for mode, key in (("ref_cpu go-shaped", "go_shaped"), ("ref_cpu tuned", "tuned")):
        m = cpu.get("modes", {}).get(key)
        if m:
            out.append("| %s | %s | %d | %.3g | — | — | pinned to oracle |" % (LABEL[cfg], mode, m["threads"], m["value"]))
    traffic = ("; PMC %.1f B/rec" % (r["traffic"] / d["config"]["records_per_gpu"])) if r.get("traffic") else ""
    out.append("| %s | HIP `%s` | 1 GPU | %.3g | %.0f kernel (%.3f ms) | %.1f %% kernel, %.1f %% step%s | bit-exact (tests) |" % (
        LABEL[cfg], r["kernel"].split("<")[0] if "+" not in r["kernel"] else "sketch pass", d["value"],
        r["achieved"], r["kernel_ms"], 100 * r["frac"],
        100 * r["step_bytes_per_record"] * d["config"]["records_per_gpu"] / (d["ms_per_step"] * 1e-3) / 8e12,
        traffic))
    pr = d.get("production")
    if pr:
        out.append("| %s | HIP, device-resident %s-record launches (Go batch) | 1 GPU | %.3g | — | %.1f %% kernel | — |" % (
            LABEL[cfg], pow2(pr.get("batch_records", 1 << 20)), pr["records_per_s"], 100 * pr["kernel_frac"]))
    hf = d.get("host_fed")
    if hf:
        out.append("| %s | HIP, host-fed %s-record pinned batches (PCIe H2D incl.) | 1 GPU | %.3g | — | PCIe-bound | — |" % (
            LABEL[cfg], pow2(hf.get("batch_records", 1 << 20)), hf["value"]))
    hr = d.get("host_fed_raw")
    if hr:
        out.append("| %s | HIP, raw 72-B samples via gpuagg_raw_feed_put, %s %d threads (PCIe incl.) | 1 GPU | %.3g | — | PCIe-bound | — |" % (
            LABEL[cfg], hr.get("feed_mode", "raw_dma"), hr.get("feed_threads", 1), hr["value"]))
        best = hr.get("best")
        if best and best["value"] > hr["value"]:
            out.append("| %s | HIP, raw samples via gpuagg_raw_feed_put, %s %d threads (PCIe incl.) | 1 GPU | %.3g | — | PCIe-bound | — |" % (
                LABEL[cfg], best["mode"], best["threads"], best["value"]))
    return out


def scrape_rows(paths):
    """Scrape cost per config: gpuagg_snapshot + gpuagg_result_render_text on the bench's state."""
    out = ["| Config | series | text MB | snapshot ms | render ms (+ copy, copying API) | % of a 15 s epoch (warm) | cold scrape ms | % (cold) |",
           "|---|---|---|---|---|---|---|---|"]
    for path in paths:
        d = json.load(open(path))
        sc = d.get("scrape")
        if not sc:
            continue
        cfg = path.rsplit("_bench_", 1)[-1].replace(".json", "")
        cold = sc.get("cold_snapshot_ms")
        out.append("| %s | %d | %.1f | %.1f | %.1f (+ %.1f) | %.2f %% | %s | %s |" % (
            LABEL[cfg], sc["series"], sc["text_bytes"] / 1e6, sc["snapshot_ms"], sc["render_ms"], sc.get("copy_ms", 0.0),
            100 * sc["epoch_frac"], "%.0f" % (cold + sc["cold_render_ms"]) if cold is not None else "—",
            "%.2f %%" % (100 * sc["cold_epoch_frac"]) if cold is not None else "—"))
    return out


if __name__ == "__main__":
    print("| Config | Mode | Cores / GPUs | records/s | GB/s (alg.) | % of 8 TB/s | Parity |")
    print("|---|---|---|---|---|---|---|")
    for p in sys.argv[1:]:
        print("\n".join(rows(p)))
    print()
    print("\n".join(scrape_rows(sys.argv[1:])))
