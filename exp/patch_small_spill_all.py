"""Experiment: small tier-1 launches (<= 2^22 records) keep no bins in LDS when GA_SPILL_ALL
is set: every dense update goes to the deferred spill lists (8 B per update, folded once
per deferral budget) instead of each workgroup loading and storing its 80 KiB staged copy
of the LDS bins per launch."""
import sys

p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
old = """    const uint32_t L4 = prefix((kLdsBytes - c->ipl_bytes - kL4ExtraBytes) / 4);"""
new = """    const uint32_t L4 = (n <= (1ull << 22) && getenv("GA_SPILL_ALL")) ? 0u
                        : prefix((kLdsBytes - c->ipl_bytes - kL4ExtraBytes) / 4);"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
