"""Markdown rows of DESIGN.md section 8 from bench lines (diagnostics helper).

    python scripts/results_table.py profiles/round2/r5b_bench_c2.json [...]
"""

import json
import sys


def row(path):
    d = json.load(open(path))
    r = d["roofline"]
    cpu = d.get("cpu_baseline", {})
    return "| %s | %d | %.3g | %.3f | `%s` | %.3f | %.1f %% | %s | %s |" % (
        path.rsplit("_bench_", 1)[-1].replace(".json", ""), d["config"]["records_per_gpu"], d["value"],
        d["ms_per_step"], r["kernel"], r["kernel_ms"], 100 * r["frac"],
        "%.1f" % (r["traffic"] / d["config"]["records_per_gpu"]) if r.get("traffic") else "—",
        "%.3g" % cpu["value"] if cpu else "—")


if __name__ == "__main__":
    print("| config | records / step | records/s | ms/step | dominant kernel | kernel ms (HIP events) "
          "| % of 8 TB/s | HBM B/rec (PMC) | CPU tuned, 16 thr |")
    print("|---|---|---|---|---|---|---|---|---|")
    for p in sys.argv[1:]:
        print(row(p))
