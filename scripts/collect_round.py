"""Copies one GPU session's evidence (scripts/gpu_check.sh TAG ...) from gpurun_out/ into
profiles/<round>/ and refreshes profiles/pmc_<config>.json from that session's PMC
summaries -- only those collected from the library build that is in the tree now.

    python scripts/collect_round.py TAG [round4]
"""

import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    tag = sys.argv[1]
    rnd = sys.argv[2] if len(sys.argv) > 2 else "round4"
    from retina_amd import build
    bid = build.build_id()
    src, dst = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    copied = []
    for pat in ("%s_bench_*.json", "%s_*_kernel_stats.csv", "%s_pytest.log", "%s_smoke.log", "%s_info.txt",
                "%s_pmc_*.json", "%s_ab.jsonl"):
        for f in glob.glob(os.path.join(src, pat % tag)):
            if os.path.getsize(f):
                shutil.copy(f, dst)
                copied.append(os.path.basename(f))
    for f in glob.glob(os.path.join(src, "%s_pmc_*.json" % tag)):
        cfg = os.path.basename(f)[len(tag) + 5:-5]
        pmc = json.load(open(f))
        if pmc.get("build_id") != bid:
            print("skip %s: build %s, tree %s" % (f, pmc.get("build_id"), bid))
            continue
        shutil.copy(f, os.path.join(ROOT, "profiles", "pmc_%s.json" % cfg))
        copied.append("pmc_%s.json" % cfg)
    for f in glob.glob(os.path.join(src, "%s_bench_*.json" % tag)):
        try:
            d = json.load(open(f))
        except ValueError:
            continue
        if d.get("build_id") != bid:
            print("note %s: build %s, tree %s" % (f, d.get("build_id"), bid))
    print("\n".join(sorted(copied)))


if __name__ == "__main__":
    main()
