"""Wide-list fold threshold experiment: fold when the fullest list reaches FRAC of its
capacity instead of half.  usage: patch_foldthr.py SRC_DIR NUM DEN"""
import sys
src, num, den = sys.argv[1], sys.argv[2], sys.argv[3]
p = src + "/gpuagg_kernels.hip"
s = open(p).read()
old = "a.fold_cond ? a.sp_cap / 2 : 0u);"
assert s.count(old) == 1
s = s.replace(old, "a.fold_cond ? (uint32_t)((uint64_t)a.sp_cap * %s / %s) : 0u);" % (num, den))
open(p, "w").write(s)
