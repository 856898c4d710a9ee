"""Probe: spill-only plans (C2, C4) defer their spill folds and staged reductions at full-size
launches too, with list space for 2^23 records per workgroup (~21 full-size C2 launches)."""
import sys
p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
old = "    const bool small_spill = c->dense_len > a.lds_bins && a.chunk * kDeferLaunches <= kMaxRecordsPerBlock;"
assert old in s
s = s.replace(old, "    const bool small_spill = c->dense_len > a.lds_bins;")
old = "    uint64_t budget = defer ? std::max<uint64_t>(a.chunk, std::min<uint64_t>(kMaxRecordsPerBlock,"
assert old in s
s = s.replace(old, "    uint64_t budget = defer ? std::max<uint64_t>(a.chunk, std::min<uint64_t>(1ull << 23,")
open(p, "w").write(s)
