"""Experiment (round 6): spill-list entries written with non-temporal stores."""
import sys

p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()
old = """    if (pos < spill_cap) {  // w < 256 and spill_cap < 2^24: 24-bit multiply
      spill[mul_u24(w, spill_cap) + pos] = entry(bin, nbytes);
      return;
    }"""
new = """    if (pos < spill_cap) {  // w < 256 and spill_cap < 2^24: 24-bit multiply
      __builtin_nontemporal_store(entry(bin, nbytes), &spill[mul_u24(w, spill_cap) + pos]);
      return;
    }"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
