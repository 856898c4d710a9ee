"""Experiment: wide_insert issues the doorkeeper atomic and both hot-cache candidates' tag
reads together (one LDS round trip), then both candidates' keys, instead of a dependent
chain door -> tag0 -> keys0 -> tag1 -> keys1."""
import sys

p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()
old = """  const uint64_t kh = key_hash(k0, k1, k2);
  bool claim = true;
  if (s.door_log2) {
    const uint32_t bit = (uint32_t)(kh >> 40) & ((1u << s.door_log2) - 1u);
    claim = (atomicOr(&s.door[bit >> 5], 1u << (bit & 31u)) >> (bit & 31u)) & 1u;
  }
  if (!(s.hot_n && hot_add(s, (uint32_t)kh, k0, k1, k2, 1, b, claim))) wide_append(s, kh, k0, k1, k2, 1, b);
}"""
new = """  const uint64_t kh = key_hash(k0, k1, k2);
  if (s.hot_n) {
    const uint32_t h = (uint32_t)kh;
    HotKey *e0 = &s.hot[h & (s.hot_n - 1u)], *e1 = &s.hot[(h + 0x9E37u) & (s.hot_n - 1u)];
    unsigned long long t0 = __hip_atomic_load(&e0->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    unsigned long long t1 = __hip_atomic_load(&e1->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    uint32_t dw = ~0u, bit = 0;
    if (s.door_log2) {
      bit = (uint32_t)(kh >> 40) & ((1u << s.door_log2) - 1u);
      dw = atomicOr(&s.door[bit >> 5], 1u << (bit & 31u));
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // keys read after the tags
    const unsigned long long a0 = e0->k0, a1 = e0->k1, a2 = e0->k2;
    const unsigned long long c0 = e1->k0, c1 = e1->k1, c2 = e1->k2;
    HotKey *hit = nullptr;
    if (t0 == 2ULL && a0 == k0 && a1 == k1 && a2 == k2) hit = e0;
    else if (t1 == 2ULL && c0 == k0 && c1 == k1 && c2 == k2) hit = e1;
    if (hit) {
      atomicAdd(&hit->cnt, 1ULL);
      if (b) atomicAdd(&hit->byt, (unsigned long long)b);
      return;
    }
    if ((dw >> (bit & 31u)) & 1u) {  // second sighting: claim a free candidate
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        HotKey *e = q ? e1 : e0;
        if ((q ? t1 : t0) == 0ULL && atomicCAS(&e->tag, 0ULL, 1ULL) == 0ULL) {
          e->k0 = k0;
          e->k1 = k1;
          e->k2 = k2;
          e->cnt = 1ULL;
          e->byt = b;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __hip_atomic_store(&e->tag, 2ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          return;
        }
      }
    }
  }
  wide_append(s, kh, k0, k1, k2, 1, b);
}"""
assert old in s
open(p, "w").write(s.replace(old, new))
