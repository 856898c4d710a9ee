// Secondary ceilings of MI355X for the configs that are not HBM-streaming-bound
// (VERDICT r5 item 7).  Diagnostic, not the product.  One JSON line per case:
//   stream4   4 u32 columns, 16-byte non-temporal loads, the next step prefetched (the
//             tier-1 kernel's skeleton): 1 x 1024-thread workgroup per CU (its geometry) and
//             4 per CU (no LDS limit) -> the streaming ceiling of that access pattern
//   lds_add   random u32 adds into a 64 KiB LDS array (ds_add_u32; "rtn": result used),
//             and the conflict-free pattern (lane-consecutive words) for the bank cost
//   lds_add64 random u64 adds (ds_add_u64) / lds_cas64: one u64 CAS attempt (ds_cmpst_b64)
//   gather    random 4-byte loads from a table of T bytes (8 independent per lane per step)
//   gatomic   random u32 global atomic adds (memory-side, at the L2) into T bytes
// Rates: ops/s chip-wide (lane operations), wave-instructions/s = ops/s / 64.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mbb scripts/microbench_bounds.hip && /tmp/mbb
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ uint32_t xs(uint32_t &s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}

__device__ __forceinline__ uint32_t seed_of() {
  return (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u + 0x9E3779B9u;
}

__device__ __forceinline__ uint4 nt_ld(const uint4 *p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_nontemporal_load((const v4u *)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// 4 columns of nvec uint4, contiguous chunk per workgroup, next step prefetched
__global__ __launch_bounds__(1024) void stream4(const uint4 *a, const uint4 *b, const uint4 *c, const uint4 *d,
                                                uint64_t nvec, uint32_t *out) {
  const uint64_t chunk = (nvec + gridDim.x - 1) / gridDim.x;
  const uint64_t v0 = blockIdx.x * chunk, v1 = v0 + chunk < nvec ? v0 + chunk : nvec;
  uint32_t acc = 0;
  uint64_t v = v0 + threadIdx.x;
  if (v < v1) {
    uint4 na = nt_ld(&a[v]), nb = nt_ld(&b[v]), nc = nt_ld(&c[v]), nd = nt_ld(&d[v]);
    for (; v < v1; v += blockDim.x) {
      const uint4 xa = na, xb = nb, xc = nc, xd = nd;
      const uint64_t w = v + blockDim.x < v1 ? v + blockDim.x : v;
      na = nt_ld(&a[w]);
      nb = nt_ld(&b[w]);
      nc = nt_ld(&c[w]);
      nd = nt_ld(&d[w]);
      acc += xa.x ^ xb.y ^ xc.z ^ xd.w ^ xa.w ^ xb.x ^ xc.y ^ xd.z;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;  // keeps the loads
}

// kPat 0: random over the 64 KiB array; 1: lane-consecutive (conflict-free)
template <bool kRtn, int kPat>
__global__ __launch_bounds__(1024) void lds_add(uint32_t iters, uint32_t *out) {
  __shared__ uint32_t bins[16384];
  for (uint32_t i = threadIdx.x; i < 16384; i += blockDim.x) bins[i] = 0;
  __syncthreads();
  uint32_t s = seed_of(), acc = 0;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t idx = kPat == 0 ? (xs(s) & 16383u) : (((wave * 8 + j + it) & 255u) << 6 | lane);
      if (kRtn)
        acc += __hip_atomic_fetch_add(&bins[idx], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else
        __hip_atomic_fetch_add(&bins[idx], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
  const uint32_t r = bins[threadIdx.x] + acc;
  if (r == 0x12345678u) out[0] = r;
}

// kOp 0: ds_add_u64 random; 1: one ds_cmpst_b64 attempt (expects 0) random
template <int kOp>
__global__ __launch_bounds__(1024) void lds_64(uint32_t iters, uint32_t *out) {
  __shared__ unsigned long long bins[8192];
  for (uint32_t i = threadIdx.x; i < 8192; i += blockDim.x) bins[i] = 0;
  __syncthreads();
  uint32_t s = seed_of();
  unsigned long long acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t idx = xs(s) & 8191u;
      if (kOp == 0)
        __hip_atomic_fetch_add(&bins[idx], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else
        acc += atomicCAS(&bins[idx], 0ull, (unsigned long long)s);
    }
  }
  __syncthreads();
  const unsigned long long r = bins[threadIdx.x] + acc;
  if (r == 0x12345678ull) out[0] = (uint32_t)r;
}

// 8 independent random 4-byte loads per lane per step from t[0, mask]
__global__ __launch_bounds__(256) void gather(const uint32_t *t, uint32_t mask, uint32_t iters, uint32_t *out) {
  uint32_t s = seed_of(), acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = t[xs(s) & mask];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// random non-returning global atomic adds (memory-side) into t[0, mask]
__global__ __launch_bounds__(256) void gatomic(uint32_t *t, uint32_t mask, uint32_t iters) {
  uint32_t s = seed_of();
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) atomicAdd(&t[xs(s) & mask], 1u);
  }
}

__global__ void fill(uint32_t *p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i * 2654435761u ^ seed;
}

template <class F>
static float time_ms(F launch, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();  // warm-up
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / reps;
}

static void line(const char *name, const char *extra, double ms, double ops, const char *unit_note) {
  printf("{\"case\": \"%s\"%s, \"ms\": %.4f, \"ops\": %.0f, \"ops_per_s\": %.4g, \"wave_insts_per_s\": %.4g, "
         "\"note\": \"%s\"}\n",
         name, extra, ms, ops, ops / (ms * 1e-3), ops / 64.0 / (ms * 1e-3), unit_note);
  fflush(stdout);
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *out;
  CK(hipMalloc(&out, 64));
  char extra[256];

  // ---- streaming: 100M records x 4 columns (1.6 GB) ----
  {
    const size_t n = 100000000, nvec = n / 4;
    uint32_t *col[4];
    for (int i = 0; i < 4; ++i) {
      CK(hipMalloc(&col[i], n * 4));
      hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, col[i], n, 77u * (i + 1));
    }
    for (int per_cu : {1, 2, 4}) {
      const int grid = cus * per_cu;
      const float ms = time_ms([&] {
        hipLaunchKernelGGL(stream4, dim3(grid), dim3(1024), 0, 0, (const uint4 *)col[0], (const uint4 *)col[1],
                           (const uint4 *)col[2], (const uint4 *)col[3], (uint64_t)nvec, out);
      }, 20);
      snprintf(extra, sizeof extra, ", \"workgroups_per_cu\": %d, \"GBps\": %.1f", per_cu, 16.0 * n / (ms * 1e-3) / 1e9);
      line("stream4", extra, ms, (double)n, "records (16 B each)");
    }
    for (int i = 0; i < 4; ++i) CK(hipFree(col[i]));
  }

  // ---- LDS atomics ----
  {
    const uint32_t iters = 4096;
    for (int per_cu : {1, 2}) {
      const int grid = cus * per_cu;
      const double ops = (double)grid * 1024 * iters * 8;
      struct C {
        const char *name;
        void (*k)(uint32_t, uint32_t *);
      } cases[] = {{"lds_add_u32_random", lds_add<false, 0>}, {"lds_add_u32_random_rtn", lds_add<true, 0>},
                   {"lds_add_u32_conflict_free", lds_add<false, 1>}, {"lds_add_u64_random", lds_64<0>},
                   {"lds_cas_u64_random", lds_64<1>}};
      for (const C &c : cases) {
        const float ms = time_ms([&] { hipLaunchKernelGGL(c.k, dim3(grid), dim3(1024), 0, 0, iters, out); }, 5);
        snprintf(extra, sizeof extra, ", \"workgroups_per_cu\": %d, \"per_cu_per_clk_at_2.4GHz\": %.3f", per_cu,
                 ops / (ms * 1e-3) / cus / 2.4e9);
        line(c.name, extra, ms, ops, "lane operations");
      }
    }
  }

  // ---- random gathers and global atomics over table sizes ----
  {
    const size_t max_words = (size_t)1 << 28;  // 1 GiB
    uint32_t *t;
    CK(hipMalloc(&t, max_words * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, t, max_words, 3u);
    const int grid = cus * 8;  // 8 x 256 threads per CU
    for (int lg : {14, 16, 18, 20, 22, 24, 26, 28}) {
      const uint32_t mask = (uint32_t)(((size_t)1 << lg) - 1);
      const uint32_t iters = 512;
      const double ops = (double)grid * 256 * iters * 8;
      const float ms = time_ms([&] { hipLaunchKernelGGL(gather, dim3(grid), dim3(256), 0, 0, t, mask, iters, out); }, 5);
      snprintf(extra, sizeof extra, ", \"table_bytes\": %zu", (size_t)4 << lg);
      line("gather_u32_random", extra, ms, ops, "4-byte loads (one L2 request each)");
    }
    for (int lg : {16, 20, 24, 28}) {
      const uint32_t mask = (uint32_t)(((size_t)1 << lg) - 1);
      const uint32_t iters = 64;
      const double ops = (double)grid * 256 * iters * 4;
      const float ms = time_ms([&] { hipLaunchKernelGGL(gatomic, dim3(grid), dim3(256), 0, 0, t, mask, iters); }, 3);
      snprintf(extra, sizeof extra, ", \"table_bytes\": %zu", (size_t)4 << lg);
      line("global_atomic_add_u32_random", extra, ms, ops, "memory-side atomics");
    }
    CK(hipFree(t));
  }
  CK(hipFree(out));
  return 0;
}
