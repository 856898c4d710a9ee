"""Diagnostics: the wide-list fold prints the fullest list (the launch's flag) and its
threshold, once per launch.  usage: patch_foldprint.py SRC_DIR"""
import sys
p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()
old = "    if (thr && atomicOr(&flag[parity], 0u) < thr) return;  // the same value for every workgroup"
assert s.count(old) == 1
s = s.replace(old, "    if (blockIdx.x == 0 && threadIdx.x == 0) printf(\"FOLDDIAG max %u thr %u cap %u\\n\", atomicOr(&flag[parity], 0u), thr, cap);\n" + old)
open(p, "w").write(s)
