"""Experiment (round 6, C2 only): the dense radix block from 2 prefix compares, not 4
(C2's pod IPs fall in 2 /16s; wrong for more -- timing only)."""
import sys

p = sys.argv[1] + "/gpuagg_internal.h"
s = open(p).read()
old = """  d = p == p3 ? d3 : d;
  d = p == p2 ? d2 : d;
  d = p == p1 ? d1 : d;"""
assert old in s
s = s.replace(old, "  d = p == p1 ? d1 : d;")
open(p, "w").write(s)
