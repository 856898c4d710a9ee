"""Experiment: the spill-window fold with one workgroup per CU (half the partitions, half
the staged partial bytes that stage_reduce_kernel reads) instead of two."""
import sys

p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
old = "g.win_blocks = nwin * std::max<uint32_t>(1u, 2u * c->n_cu / nwin);"
assert old in s
s = s.replace(old, "g.win_blocks = nwin * std::max<uint32_t>(1u, c->n_cu / nwin);")
open(p, "w").write(s)
