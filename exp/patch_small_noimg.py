"""Experiment: small launches (<= 2^22 records) without the per-workgroup LDS IP image:
GA_SMALL_NOIMG=1 drops it from the sketch pass (HBM IP-table lookups), =2 also from the
dense pass (tier 1 off: the HBM-table dense kernel), so a 2^20-record launch does not
refill 40 KiB per workgroup for 4096 records."""
import sys

p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
old = """  if (s.hll_p && c->ipl_all_bytes) {
    s.ipl = c->d_ipl_all;"""
new = """  if (s.hll_p && c->ipl_all_bytes && !(n <= (1ull << 22) && getenv("GA_SMALL_NOIMG"))) {
    s.ipl = c->d_ipl_all;"""
assert old in s
s = s.replace(old, new)
old = """  if (a.dense_ng && !a.dns_compact && c->ipl_bytes && !spans.empty() &&
      c->ipl_bytes + kL4ExtraBytes < kLdsBytes) {"""
new = """  if (a.dense_ng && !a.dns_compact && c->ipl_bytes && !spans.empty() &&
      c->ipl_bytes + kL4ExtraBytes < kLdsBytes &&
      !(n <= (1ull << 22) && getenv("GA_SMALL_NOIMG") && atoi(getenv("GA_SMALL_NOIMG")) >= 2)) {"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
