"""Experiment (round 6): sketch folds deferred across 2^SHIFT records per scatter workgroup
(product 2^20).  usage: patch_skdefer.py SRC_DIR [SHIFT]"""
import sys

src = sys.argv[1]
shift = sys.argv[2] if len(sys.argv) > 2 else "22"
p = src + "/gpuagg_runtime.cpp"
s = open(p).read()
old = "constexpr uint64_t kSketchDeferRecords = 1ull << 20;"
assert old in s
s = s.replace(old, "constexpr uint64_t kSketchDeferRecords = 1ull << %s;" % shift)
open(p, "w").write(s)
