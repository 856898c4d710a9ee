"""Summarise rocprofv3 --pmc passes into per-launch HBM traffic for one kernel (or pass).

    python scripts/pmc_summary.py OUT.json KERNEL RECORDS BUILD_ID PASS_DIR...

KERNEL is the signature bench.py reports in roofline.kernel (e.g.
"dense_lds_kernel<2, true, 41u>"); a pass of several kernels is written "a+b" and its
counters are the sum of each kernel's per-dispatch average.  Reads every
*counter_collection.csv under the pass directories and applies the gfx950 corrections of
MI355X_MICROARCH.md (HBM section): FETCH_SIZE (KiB) counts half of the bytes of wide
coalesced reads, so it is doubled; WRITE_SIZE (KiB) is taken as is.
"""

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, kernel, records, build_id, dirs = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5:]
    parts = [p for p in kernel.split("+") if p]
    vals = {p: defaultdict(list) for p in parts}
    every = defaultdict(lambda: defaultdict(list))  # every kernel of the step, by name
    names = set()
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                short = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("gpuagg::", "")
                every[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
                for p in parts:
                    if p in row["Kernel_Name"]:
                        names.add(row["Kernel_Name"])
                        vals[p][row["Counter_Name"]].append(float(row["Counter_Value"]))
    avg = defaultdict(float)
    disp = {}
    for p in parts:
        for k, v in vals[p].items():
            avg[k] += sum(v) / len(v)
            disp["%s:%s" % (p, k)] = len(v)
    res = {"kernel": sorted(names), "kernel_signature": kernel, "records_per_launch": records,
           "build_id": build_id,
           "counters_avg_per_dispatch": dict(avg), "dispatches": disp}
    if "FETCH_SIZE" in avg:
        rd = 2.0 * avg["FETCH_SIZE"] * 1024
        wr = avg.get("WRITE_SIZE", 0.0) * 1024
        res.update({"hbm_read_bytes_corrected": rd, "hbm_write_bytes": wr,
                    "hbm_bytes_per_launch_corrected": rd + wr,
                    "hbm_bytes_per_record": (rd + wr) / records,
                    "correction": "read = 2 x FETCH_SIZE (gfx950 wide-read tally); write = WRITE_SIZE"})
    if "SQ_WAVE_CYCLES" in avg and "SQ_BUSY_CYCLES" in avg:
        res["derived"] = {
            "lds_issue_stall_frac": avg.get("SQ_WAIT_INST_LDS", 0) / avg["SQ_WAVE_CYCLES"],
            "wait_any_frac": avg.get("SQ_WAIT_ANY", 0) / avg["SQ_WAVE_CYCLES"],
            "active_inst_frac": avg.get("SQ_ACTIVE_INST_ANY", 0) / avg["SQ_WAVE_CYCLES"],
        }
    if "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
        res.setdefault("derived", {})["lds_bank_conflict_frac"] = (
            avg.get("SQ_LDS_BANK_CONFLICT", 0) / avg["SQ_LDS_IDX_ACTIVE"])
    # per-kernel averages (every kernel of the step, the fold / reduce passes included), with
    # the same HBM correction, so a step's traffic can be split by kernel
    per = {}
    for k, cv in every.items():
        a = {c: sum(v) / len(v) for c, v in cv.items()}
        if "FETCH_SIZE" in a:
            a["hbm_bytes_corrected"] = 2.0 * a["FETCH_SIZE"] * 1024 + a.get("WRITE_SIZE", 0.0) * 1024
            a["hbm_bytes_per_record"] = a["hbm_bytes_corrected"] / records
        per[k] = a
    res["per_kernel"] = per
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
