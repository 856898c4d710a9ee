"""Experiment: wide-key fold segments of 2^11 slots (80 KiB of LDS: two fold workgroups per
CU, so one's segment load / store overlaps the other's inserts) -- 8192 segment lists for
a 2^24-slot table instead of 4096."""
import sys

p = sys.argv[1] + "/gpuagg_internal.h"
s = open(p).read()
for old, new in [("constexpr uint32_t kSparseSegLog2 = 13, kSparseMaxSegLists = 4096;",
                  "constexpr uint32_t kSparseSegLog2 = 13, kSparseMaxSegLists = 8192;"),
                 ("constexpr uint32_t kWideSegLog2 = 12, kWideMaxLog2 = kWideSegLog2 + 12;",
                  "constexpr uint32_t kWideSegLog2 = 11, kWideMaxLog2 = kWideSegLog2 + 13;"),
                 ('static_assert(kWideHomeShift + kWideSegLog2 == 64, "home field fills the word");',
                  'static_assert(kWideHomeShift + kWideSegLog2 <= 64, "home field fits the word");')]:
    assert old in s, old
    s = s.replace(old, new)
open(p, "w").write(s)
