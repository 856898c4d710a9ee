"""Probe: 64 GiB of wide-key lists per ctx (product: 32 GiB, at most 1/8 of the device)."""
import sys
p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
for old, new in [("constexpr uint64_t kWideListBytes = 32ull << 30;", "constexpr uint64_t kWideListBytes = 64ull << 30;"),
                 ("(uint64_t)prop.totalGlobalMem / 8);", "(uint64_t)prop.totalGlobalMem / 4);")]:
    assert old in s, old
    s = s.replace(old, new)
open(p, "w").write(s)
