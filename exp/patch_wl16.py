"""Experiment: 16 GiB of wide-key lists per context (kWideListBytes), so the conditional
fold's table pass runs less often."""
import sys

p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
old = "constexpr uint64_t kWideListBytes = 8ull << 30;"
assert old in s
open(p, "w").write(s.replace(old, "constexpr uint64_t kWideListBytes = 16ull << 30;"))
