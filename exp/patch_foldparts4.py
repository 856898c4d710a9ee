"""Probe: spill-window fold with 4 partitions per window (product: 2 x CUs / windows, 25 at C2)."""
import sys
p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
old = "g.win_blocks = nwin * std::max<uint32_t>(1u, 2u * c->n_cu / nwin);"
assert old in s
open(p, "w").write(s.replace(old, "g.win_blocks = nwin * 4;"))
