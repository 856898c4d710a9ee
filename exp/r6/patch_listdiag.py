"""Diagnostics: one line per full segment list at the end of an aggregation launch
(wide_kernel / aggregate_kernel sp_counts_out).  usage: patch_listdiag.py SRC_DIR"""
import sys
p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()
old = """    a.sp_counts[(size_t)blockIdx.x * a.sp_nwin + w] = c;"""
new = old + """
    if (c >= a.sp_cap) printf("LISTDIAG wg %u seg %u raw %u\\n", blockIdx.x, w, sctr[w]);"""
assert s.count(old) == 1
s = s.replace(old, new)
open(p, "w").write(s)
