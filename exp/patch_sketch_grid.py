"""Experiment: small sketch launches (<= 2^22 records) on n_cu / GA_SK_DIV scatter
workgroups (env, default 1): each workgroup's LDS image fill and ring flushes are spread
over more records."""
import sys

p = sys.argv[1] + "/gpuagg_runtime.cpp"
s = open(p).read()
old = """  s.blocks = c->n_cu;
  s.win_shift"""
new = """  s.blocks = c->n_cu;
  if (n <= (1ull << 22) && getenv("GA_SK_DIV")) s.blocks = std::max<uint32_t>(8u, c->n_cu / (uint32_t)atoi(getenv("GA_SK_DIV")));
  s.win_shift"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
