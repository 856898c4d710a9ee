"""Probe (valid only for <= 4 radix prefixes, as C5's pods have): the prefix compare loop of
radix_block runs 4 iterations instead of kRadixSmall (8)."""
import sys
p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()
old = "  for (uint32_t j = 0; j < kRadixSmall; ++j)\n    b = (j < t.rpn && lo"
assert old in s
open(p, "w").write(s.replace(old, "  for (uint32_t j = 0; j < 4; ++j)\n    b = (j < t.rpn && lo"))
