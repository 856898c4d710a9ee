"""Probe: device-conditional wide-list folds at threshold a.sp_cap / 4 (product: sp_cap / 2)."""
import sys
p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()
old = "a.fold_cond ? a.sp_cap / 2 : 0u"
assert old in s
open(p, "w").write(s.replace(old, "a.fold_cond ? a.sp_cap / 4 : 0u"))
