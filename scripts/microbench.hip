// Ceilings for the aggregation loop on MI355X (diagnostic; not part of the product).
// Streams 4 u32 columns of N records (16 B/record) and adds IP-table gathers:
//   stream      : loads only
//   gather2x8   : + 2 independent 8-byte gathers per IP (cuckoo, 2 IPs/record)
//   gather1x8   : + 1 8-byte gather per IP
//   gather1x16  : + 1 16-byte gather per IP (2-entry bucket)
//   lds2        : gather1x16 + 2 LDS u64 atomics per record into a 160 KB window
// for several launch geometries. Prints one JSON line per case.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mb scripts/microbench.hip && /tmp/mb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                       \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ uint32_t h1(uint32_t x) {
  x ^= x >> 16;
  const uint32_t h = x * 0x9E3779B1u;
  return h ^ (h >> 15);
}
__device__ __forceinline__ uint32_t h2(uint32_t x) {
  x ^= x >> 16;
  const uint32_t h = x * 0x85EBCA77u;
  return h ^ (h >> 13);
}

template <int MODE>
__global__ __launch_bounds__(1024) void kern(const uint4 *a, const uint4 *b, const uint4 *c,
                                             const uint4 *d, size_t nvec, const uint64_t *tab,
                                             uint32_t mask, unsigned long long *out) {
  extern __shared__ unsigned long long win[];
  if (MODE == 4) {
    for (uint32_t i = threadIdx.x; i < 20480; i += blockDim.x) win[i] = 0;
    __syncthreads();
  }
  const size_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const size_t s = blockIdx.x * per, e = s + per < nvec ? s + per : nvec;
  unsigned long long acc = 0;
  for (size_t v = s + threadIdx.x; v < e; v += blockDim.x) {
    const uint4 x = a[v], y = b[v], z = c[v], w = d[v];
    acc += x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w ^ z.x ^ z.y ^ z.z ^ z.w ^ w.x ^ w.y ^ w.z ^ w.w;
    if (MODE >= 1) {
      const uint32_t ip[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
      uint64_t r[8];
      if (MODE == 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = tab[h1(ip[k]) & mask] ^ tab[h2(ip[k]) & mask];
      } else if (MODE == 2) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = tab[h1(ip[k]) & mask];
      } else {
        const uint4 *t4 = (const uint4 *)tab;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint4 q = t4[(h1(ip[k]) & mask) >> 1];
          r[k] = ((uint32_t)q.x == ip[k]) ? q.y : q.w;
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += r[k];
      if (MODE == 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          atomicAdd(&win[(uint32_t)r[k] % 20000u], (1ULL << 44) | z.x);
          atomicAdd(&win[(uint32_t)r[k + 4] % 20000u], (1ULL << 44) | z.y);
        }
      }
    }
  }
  if (MODE == 4) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 20000; i += blockDim.x) acc += win[i];
  }
  atomicAdd(out, acc);
}

__global__ void fill(uint32_t *p, size_t n, uint32_t seed, uint32_t pod_mod) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = pod_mod ? (10u | ((x % pod_mod) << 8)) : x;
  }
}

int main() {
  const size_t n = 100000000, nvec = n / 4;
  uint32_t *col[4];
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&col[i], n * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, col[i], n, 77u * (i + 1), i < 2 ? 10000u : 0u);
  }
  unsigned long long *out;
  CK(hipMalloc(&out, 8));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  struct G { int blocks, threads; };
  const G geos[] = {{ncu, 1024}, {ncu * 2, 512}, {ncu * 4, 256}, {ncu * 8, 256}};
  const uint32_t tabsz[] = {4096, 32768, 262144};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode <= 4; ++mode) {
    for (uint32_t ts : tabsz) {
      if (mode == 0 && ts != 4096) continue;
      uint64_t *tab;
      CK(hipMalloc(&tab, ts * 8));
      hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, 0, (uint32_t *)tab, (size_t)ts * 2, 5u, 0u);
      for (const G &g : geos) {
        if (mode == 4 && g.threads != 1024) continue;
        const size_t lds = mode == 4 ? 20480 * 8 : 0;
        auto launch = [&]() {
          switch (mode) {
            case 0: hipLaunchKernelGGL(kern<0>, dim3(g.blocks), dim3(g.threads), lds, 0, (uint4 *)col[0], (uint4 *)col[1], (uint4 *)col[2], (uint4 *)col[3], nvec, tab, ts - 1, out); break;
            case 1: hipLaunchKernelGGL(kern<1>, dim3(g.blocks), dim3(g.threads), lds, 0, (uint4 *)col[0], (uint4 *)col[1], (uint4 *)col[2], (uint4 *)col[3], nvec, tab, ts - 1, out); break;
            case 2: hipLaunchKernelGGL(kern<2>, dim3(g.blocks), dim3(g.threads), lds, 0, (uint4 *)col[0], (uint4 *)col[1], (uint4 *)col[2], (uint4 *)col[3], nvec, tab, ts - 1, out); break;
            case 3: hipLaunchKernelGGL(kern<3>, dim3(g.blocks), dim3(g.threads), lds, 0, (uint4 *)col[0], (uint4 *)col[1], (uint4 *)col[2], (uint4 *)col[3], nvec, tab, ts - 1, out); break;
            case 4: hipLaunchKernelGGL(kern<4>, dim3(g.blocks), dim3(g.threads), lds, 0, (uint4 *)col[0], (uint4 *)col[1], (uint4 *)col[2], (uint4 *)col[3], nvec, tab, ts - 1, out); break;
          }
        };
        if (mode == 4) CK(hipFuncSetAttribute((const void *)kern<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 10; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 10;
        const char *names[] = {"stream", "gather2x8", "gather1x8", "gather1x16", "lds2"};
        printf("{\"mode\": \"%s\", \"table_entries\": %u, \"blocks\": %d, \"threads\": %d, \"ms\": %.4f, "
               "\"GBps_16B\": %.1f, \"Grec_s\": %.1f}\n",
               names[mode], ts, g.blocks, g.threads, ms, 16.0 * n / (ms * 1e-3) / 1e9, n / (ms * 1e-3) / 1e9);
        fflush(stdout);
      }
      CK(hipFree(tab));
    }
  }
  return 0;
}
