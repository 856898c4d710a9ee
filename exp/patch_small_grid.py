"""Experiment: small tier-1 launches (<= 2^22 records, e.g. the Go plugin's 2^20) on
n_cu / GA_SMALL_DIV workgroups (env, default 1), so each workgroup's fixed cost (LDS image
fill, staged bin copy in / out) is spread over more records."""
import sys

p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
old = """  a.blocks = wide ? c->n_cu : c->n_cu * 4;"""
new = """  a.blocks = wide ? c->n_cu : c->n_cu * 4;
  if (a.tier1 && n <= (1ull << 22) && getenv("GA_SMALL_DIV"))
    a.blocks = std::max<uint32_t>(8u, a.blocks / (uint32_t)atoi(getenv("GA_SMALL_DIV")));"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
