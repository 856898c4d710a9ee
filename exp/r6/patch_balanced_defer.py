"""Wide-list fold: lanes balanced over the segment's concatenated lists (64-entry chunks
round-robin over the waves) and a per-segment fold decision (only segments with a list at
the threshold fold; the others keep their lists).  usage: patch_balanced_defer.py SRC_DIR"""
import sys
p = sys.argv[1] + "/gpuagg_kernels.hip"
s = open(p).read()
old = '''  uint32_t any = 0;
  for (uint32_t l = threadIdx.x; l < n_lists; l += blockDim.x) any |= counts[(size_t)l * nwin + w];
  // (a flag word in the segment's LDS: __syncthreads_or would take static LDS beyond the
  // 160 KiB the segment may fill)
  if (threadIdx.x == 0) seg[0] = 0ULL;
  __syncthreads();
  if (any) seg[0] = 1ULL;'''
new = '''  uint32_t mx = 0;
  for (uint32_t l = threadIdx.x; l < n_lists; l += blockDim.x) mx = max(mx, counts[(size_t)l * nwin + w]);
  if (threadIdx.x == 0) seg[0] = 0ULL;
  __syncthreads();
  if (thr ? mx >= thr : mx != 0u) seg[0] = 1ULL;'''
assert s.count(old) == 1
s = s.replace(old, new)
old = '''           a1.y & ((1ULL << kWideCountShift) - 1));
  };
  for (uint32_t l0 = 0; l0 < n_lists; l0 += lists_per_round) {'''
new = '''           a1.y & ((1ULL << kWideCountShift) - 1));
  };
  const uint32_t ew = s.narrow ? kWideNarrowWords : kWideEntryWords;
  if (n_lists <= 256) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    uint32_t inc[4], tot = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t l = lane * 4u + (uint32_t)q;
      const uint32_t c = l < n_lists ? counts[(size_t)l * nwin + w] : 0u;
      tot += c < cap ? c : cap;
      inc[q] = tot;
    }
    uint32_t x = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      x += lane >= (uint32_t)o ? y : 0u;
    }
    const uint32_t B = x - tot, E = (uint32_t)__shfl((int)x, 63);
    const uint32_t nchunk = (E + 63u) >> 6;
    auto locate = [&](uint32_t j0, bool valid) -> const unsigned long long * {
      const uint32_t j = j0 + lane;
      uint32_t L = (uint32_t)__popcll(__ballot(B <= j0)) - 1u;
      for (;;) {
        const uint32_t nb = (uint32_t)__shfl((int)B, (int)(L < 63u ? L + 1u : 63u));
        const bool adv = valid && L < 63u && nb <= j;
        if (!__any(adv)) break;
        L += adv ? 1u : 0u;
      }
      const uint32_t off = j - (uint32_t)__shfl((int)B, (int)L);
      const uint32_t e0 = (uint32_t)__shfl((int)inc[0], (int)L), e1 = (uint32_t)__shfl((int)inc[1], (int)L),
                     e2 = (uint32_t)__shfl((int)inc[2], (int)L);
      const uint32_t q = (off >= e0 ? 1u : 0u) + (off >= e1 ? 1u : 0u) + (off >= e2 ? 1u : 0u);
      const uint32_t st = q == 0u ? 0u : q == 1u ? e0 : q == 2u ? e1 : e2;
      return lists + (((size_t)(L * 4u + q) * nwin + w) * cap + (off - st)) * ew;
    };
    for (uint32_t c0 = wv; c0 < nchunk; c0 += 4 * nwv) {
      unsigned long long v[4][4];
      bool ok[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t c = c0 + (uint32_t)q * nwv;
        ok[q] = c < nchunk && c * 64u + lane < E;
        const unsigned long long *e = locate(c * 64u, ok[q]);
        if (ok[q]) {
          if (s.narrow) {
            v[q][0] = e[0];
            const uint64_t n = e[1];
            v[q][1] = wide_unpack1(n);
            v[q][2] = wide_unpack2(n);
            v[q][3] = e[2];
          } else {
            const ulonglong2 a0 = ((const ulonglong2 *)e)[0], a1 = ((const ulonglong2 *)e)[1];
            v[q][0] = a0.x;
            v[q][1] = a0.y;
            v[q][2] = a1.x;
            v[q][3] = a1.y;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (ok[q]) ins(make_ulonglong2(v[q][0], v[q][1]), make_ulonglong2(v[q][2], v[q][3]));
    }
  } else
  for (uint32_t l0 = 0; l0 < n_lists; l0 += lists_per_round) {'''
assert s.count(old) == 1
s = s.replace(old, new)
open(p, "w").write(s)
