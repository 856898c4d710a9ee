"""Experiment (reverse): sparse_fold_wide_kernel without the read-first fast path (every
insert starts with the CAS on K0, as in round 3)."""
import re
import sys

p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()
i = s.index("    {  // the key already sits published in its home slot")
j = s.index("    for (uint32_t probe = 0; probe < N; ++probe) {", i)
s = s[:i] + s[j:]
open(p, "w").write(s)
i = s.index("    // the key already in its home slot (a key is published whole by its claiming CAS):")
j = s.index("    for (uint32_t probe = 0; probe <= smask; ++probe) {", i)
s = s[:i] + s[j:]
open(p, "w").write(s)
