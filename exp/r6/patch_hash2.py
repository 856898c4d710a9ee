"""Cheaper group-by key hash: one fmix64 over k0 ^ k1*C1 ^ k2*C2 instead of three chained
fmix64 (timing + parity experiment).  usage: patch_hash2.py SRC_DIR"""
import sys
p = sys.argv[1] + "/gpuagg_internal.h"
s = open(p).read()
old = "  return fmix64(k0 ^ fmix64(k1 ^ fmix64(k2 ^ 0x243F6A8885A308D3ULL)));"
assert s.count(old) == 1
s = s.replace(old, "  return fmix64(k0 ^ (k1 * 0x9E3779B97F4A7C15ULL) ^ (k2 * 0xC2B2AE3D27D4EB4FULL));")
open(p, "w").write(s)
