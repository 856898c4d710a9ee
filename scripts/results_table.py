"""Markdown rows of DESIGN.md section 8 from bench lines (diagnostics helper).

    python scripts/results_table.py profiles/round2/r5b_bench_c2.json [...]
"""

import json
import sys


def row(path):
    d = json.load(open(path))
    r = d["roofline"]
    n = d["config"]["records_per_gpu"]
    cpu = d.get("cpu_baseline", {})
    step = 100 * r["step_bytes_per_record"] * n / (d["ms_per_step"] * 1e-3) / 8e12
    prod = d.get("production", {})
    sc = d.get("scrape", {})
    return "| %s | %d | %.3g | %.3f | `%s` | %.3f | %.1f %% | %.1f %% | %s | %s | %s | %s |" % (
        path.rsplit("_bench_", 1)[-1].replace(".json", ""), n, d["value"],
        d["ms_per_step"], r["kernel"], r["kernel_ms"], 100 * r["frac"], step,
        "%.1f" % (r["traffic"] / n) if r.get("traffic") else "—",
        "%.3g" % prod["records_per_s"] if prod else "—",
        "%.0f + %.0f" % (sc["snapshot_ms"], sc["render_ms"]) if sc else "—",
        "%.3g" % cpu["value"] if cpu else "—")


if __name__ == "__main__":
    print("| config | records / step | records/s | ms/step | dominant kernel | kernel ms (HIP events) "
          "| kernel % of 8 TB/s | step % | HBM B/rec (PMC) | Go-batch launches (2^22), records/s "
          "| scrape ms (snapshot + render) | CPU tuned, 16 thr |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for p in sys.argv[1:]:
        print(row(p))
