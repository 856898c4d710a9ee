"""Experiment (reverse): small spill-only launches sum their tier-1 copies per launch (round 3)
instead of accumulating them for the deferred fold."""
import sys

p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
old = "a.stage_defer = a.defer_folds && small_spill"
assert old in s
s = s.replace(old, "a.stage_defer = false && a.defer_folds && small_spill")
open(p, "w").write(s)
