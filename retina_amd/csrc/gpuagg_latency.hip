// Node-apiserver latency on the GPU: the TTL join of pkg/module/metrics/latency.go.
//
// Reference (per flow, one goroutine): ProcessFlow (:178-201) keeps TCP flows with a
// non-zero TCP id (TSval on TO_NETWORK, TSecr on FROM_NETWORK, packetparser_linux.go:
// 622-628) whose source or destination is an apiserver IP; calculateLatency (:256-305)
// inserts {src, dst, sport, dport, id} -> (Time.Nanos, flags) on TO_NETWORK unless the key
// is present, and on FROM_NETWORK looks up the mirrored key, observes round(dNanos / 1e6)
// ms, observes the handshake latency for a SYN answered by SYN+ACK, and deletes the key;
// entries that outlive the 500 ms TTL count one no_response (:123-131).
//
// Batch form (oracle/latency.py states it): the clock is the running maximum of the
// record times; an entry expires before the first record whose clock passes its expiry.
// The join is independent per key, so the batch is processed as
//   1. lat_count_kernel   per-unit (one wave's record range) event count and max time;
//   2. lat_scan_kernel    exclusive scans of both (one workgroup), batch end clock;
//   3. lat_emit_kernel    events in record order, each with its clock (wave scans),
//                         only for units that hold events;
//      lat_carry_kernel   entries still pending from earlier batches go first;
//   4. rocprim radix sort of the events by key hash (stable: record order per key);
//   5. lat_walk_kernel    one lane per key runs the TTL-cache state machine over its
//                         events and books histogram buckets / no_response with atomics;
//                         live entries carry over to the next batch.
// The ttlcache (jellydator/ttlcache v3.3.0) also touches a key on every Get hit (a repeated
// request keeps its entry alive: expiry = now + TTL, front of the LRU list) and holds at
// most LIMIT = 100000 entries: a Set at capacity evicts the least recently touched one,
// without counting it.  The capacity couples the keys, so before step 5 a first walk
// (kPass 0) books every entry's life as +1 / -1 at event positions, a scan gives the live
// count before each event and its maximum; while it stays within the limit (the normal
// case) the keys are independent and step 5 is exact, else the host replays the batch in
// event order with an LRU queue (gpuagg_runtime.cpp lat_serial_host: exact, rare; it was a
// one-thread kernel until round 5, 1.7 s per capacity-bound 2^20-record batch,
// profiles/round5/r5l_lat_serial.jsonl).
// Latency traffic is a small share of a node's records; the filter pass (1, 3) streams
// 36 B per record (src, dst, meta, ports, tcp_id, time_ns).
#include <cstring>  // rocprim's texture iterator uses memset

#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include "gpuagg_internal.h"
#include "gpuagg_launch.h"

namespace gpuagg {

constexpr uint32_t kLatThreads = 256;
constexpr uint32_t kRoleReq = 1, kRoleRep = 2, kRoleCarry = 3;

__device__ __forceinline__ bool lat_is_api(const uint32_t *api, uint32_t n_api, uint32_t ip) {
  bool hit = false;
  for (uint32_t i = 0; i < n_api; ++i) hit |= api[i] == ip;
  return hit;
}

// Event role of record i (0: not a latency event).  ToFlow gives L4 TCP for protocol 6
// (flow_utils.go:42-62); the observation point is meta bits 30-31.
__device__ __forceinline__ uint32_t lat_role(const LatArgs &a, const uint32_t *api, size_t i) {
  const uint32_t m = a.meta[i];
  if ((m & 0xFFu) != 6u || a.tcp_id[i] == 0u) return 0u;
  const uint32_t obs = m >> 30;
  const uint32_t role = obs == 3u ? kRoleReq : obs == 2u ? kRoleRep : 0u;
  if (!role) return 0u;
  return (lat_is_api(api, a.n_api, a.src[i]) || lat_is_api(api, a.n_api, a.dst[i])) ? role : 0u;
}

__device__ __forceinline__ uint64_t lat_hash(uint64_t k0, uint64_t k1) {
  return fmix64(k0 ^ fmix64(k1 ^ 0x9E3779B97F4A7C15ULL));
}

// The unit of the front end is one wave over a contiguous record range (a.chunk rows):
// the count pass reads meta, tcp_id and time for every row (src / dst only for TCP rows
// with a TCP id at observation point 2 or 3), the scan gives each unit its first event
// slot and incoming clock, and the emit pass revisits only units that hold events.
__global__ __launch_bounds__(kLatThreads) void lat_count_kernel(LatArgs a) {
  __shared__ uint32_t api[kLatMaxApi];
  if (threadIdx.x < a.n_api) api[threadIdx.x] = a.api[threadIdx.x];
  __syncthreads();
  const uint32_t u = blockIdx.x * (kLatThreads / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (u >= a.blocks) return;
  const size_t lo = min((size_t)u * a.chunk, a.n), hi = min(lo + a.chunk, a.n);  // (chunks round up)
  uint32_t cnt = 0;
  unsigned long long mx = 0;
  size_t i0 = lo;
  if (a.vec) {  // 4 rows per lane: 16-byte loads of meta / tcp_id, 2 x 16 bytes of time
    const uint4 *m4 = (const uint4 *)a.meta, *t4 = (const uint4 *)a.tcp_id;
    const ulonglong2 *c2 = (const ulonglong2 *)a.time_ns;
    const size_t hi4 = lo + ((hi - lo) & ~(size_t)3);
    for (size_t j = lo + 4 * lane; j < hi4; j += 256) {
      const uint4 m = m4[j >> 2], t = t4[j >> 2];
      const ulonglong2 c0 = c2[j >> 1], c1 = c2[(j >> 1) + 1];
      mx = max(mx, max(max(c0.x, c0.y), max(c1.x, c1.y)));
      const uint32_t mm[4] = {m.x, m.y, m.z, m.w}, tt[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int q = 0; q < 4; ++q)  // rows that can be events check the IPs (rare)
        if ((mm[q] & 0xFFu) == 6u && tt[q] != 0u && (mm[q] >> 30) >= 2u) cnt += lat_role(a, api, j + q) != 0u;
    }
    i0 = hi4;
  }
  for (size_t i = i0 + lane; i < hi; i += 64) {
    cnt += lat_role(a, api, i) != 0u;
    mx = max(mx, (unsigned long long)a.time_ns[i]);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    cnt += __shfl_xor(cnt, o);
    mx = max(mx, (unsigned long long)__shfl_xor(mx, o));
  }
  if (lane == 0) {
    a.blk_cnt[u] = cnt;
    a.blk_max[u] = mx;
  }
}

// One 1024-thread workgroup: exclusive scans (event count, clock max) over the units.
__global__ __launch_bounds__(1024) void lat_scan_kernel(LatArgs a) {
  __shared__ uint64_t s_cnt[1024];
  __shared__ unsigned long long s_max[1024];
  unsigned long long *st = a.state;
  const uint32_t per = (a.blocks + 1023) / 1024, u0 = threadIdx.x * per, u1 = min(u0 + per, a.blocks);
  uint64_t c = 0;
  unsigned long long m = 0;
  for (uint32_t u = u0; u < u1; ++u) {
    c += a.blk_cnt[u];
    m = max(m, a.blk_max[u]);
  }
  s_cnt[threadIdx.x] = c;
  s_max[threadIdx.x] = m;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive scans
    const uint64_t yc = threadIdx.x >= o ? s_cnt[threadIdx.x - o] : 0;
    const unsigned long long ym = threadIdx.x >= o ? s_max[threadIdx.x - o] : 0;
    __syncthreads();
    s_cnt[threadIdx.x] += yc;
    s_max[threadIdx.x] = max(s_max[threadIdx.x], ym);
    __syncthreads();
  }
  uint64_t base = st[kLatPending] + (threadIdx.x ? s_cnt[threadIdx.x - 1] : 0);  // carried entries first
  unsigned long long clk = max((unsigned long long)st[kLatClock], threadIdx.x ? s_max[threadIdx.x - 1] : 0ULL);
  for (uint32_t u = u0; u < u1; ++u) {
    a.blk_base[u] = base;
    a.blk_clk[u] = clk;
    base += a.blk_cnt[u];
    clk = max(clk, a.blk_max[u]);
  }
  __syncthreads();  // every thread has read st[kLatPending] / st[kLatClock]
  if (threadIdx.x == 1023) {
    st[kLatEvents] = base;
    st[kLatClockEnd] = clk;
    st[kLatCarryOut] = 0ULL;
  }
}

// Events of one unit in record order, each with clock = max time of the rows up to it
// (wave scans: max via shuffles, ranks via ballot); units without events return at once.
__global__ __launch_bounds__(kLatThreads) void lat_emit_kernel(LatArgs a) {
  __shared__ uint32_t api[kLatMaxApi];
  if (threadIdx.x < a.n_api) api[threadIdx.x] = a.api[threadIdx.x];
  __syncthreads();
  const uint32_t u = blockIdx.x * (kLatThreads / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (u >= a.blocks || a.blk_cnt[u] == 0) return;
  const size_t lo = min((size_t)u * a.chunk, a.n), hi = min(lo + a.chunk, a.n);  // (chunks round up)
  uint64_t base = a.blk_base[u];
  unsigned long long clk = a.blk_clk[u];
  // events are numbered across batches: position e of this batch (carried entries first)
  const uint64_t seq0 = a.state[kLatSeqBase] - a.state[kLatPending];
  for (size_t r = lo; r < hi; r += 64) {
    const size_t i = r + lane;
    const bool in = i < hi;
    const uint32_t role = in ? lat_role(a, api, i) : 0u;
    const unsigned long long t = in ? (unsigned long long)a.time_ns[i] : 0ULL;
    unsigned long long m = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long y = __shfl_up(m, o);
      if (lane >= (uint32_t)o) m = max(m, y);
    }
    const uint64_t ball = __ballot(role != 0u);
    if (role) {
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(ball >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ball, 0u));
      const unsigned long long c = max(clk, m);
      const uint32_t s = a.src[i], d = a.dst[i], p = a.ports[i];
      const uint64_t id = a.tcp_id[i];
      const uint32_t sp = p & 0xFFFFu, dp = p >> 16;
      // request key {src, dst, sport, dport, id}; a reply looks up the mirrored key
      const uint64_t k0 = role == kRoleReq ? ((uint64_t)s | ((uint64_t)d << 32)) : ((uint64_t)d | ((uint64_t)s << 32));
      const uint64_t k1 = role == kRoleReq ? ((uint64_t)sp | ((uint64_t)dp << 16) | (id << 32))
                                           : ((uint64_t)dp | ((uint64_t)sp << 16) | (id << 32));
      const uint32_t m8 = a.meta[i], verdict = (m8 >> 8) & 0xFFu, flags = (m8 >> 21) & 0x3Fu;
      // AddTCPFlags: packetparser sets them on every TCP flow (forwarded); SYN bit 1, ACK bit 4
      const bool has_flags = verdict == kVerdictForwarded || verdict == kVerdictRetrans;
      const uint32_t bits = role | ((has_flags && (flags & 2u)) ? 4u : 0u) | ((has_flags && (flags & 16u)) ? 8u : 0u);
      const uint64_t e = base + rank;
      a.ev[e] = LatEvent{k0, k1, c, seq0 + e, (uint32_t)((uint64_t)a.time_ns[i] % 1000000000ULL), bits};
      a.hash_in[e] = lat_hash(k0, k1);
      a.idx_in[e] = (uint32_t)e;
    }
    base += (uint64_t)__popcll(ball);
    clk = max(clk, (unsigned long long)__shfl(m, 63));
  }
}

__global__ void lat_carry_kernel(LatArgs a) {
  const uint64_t n = a.state[kLatPending];
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < n; e += (uint64_t)gridDim.x * blockDim.x) {
    const LatEvent c = a.carry_in[e];
    a.ev[e] = c;
    a.hash_in[e] = lat_hash(c.k0, c.k1);
    a.idx_in[e] = (uint32_t)e;
  }
}

// Histogram bucket of an integer latency (LinearBuckets(0, 0.5, 10): le 0, 0.5, ..., 4.5).
__device__ __forceinline__ uint32_t lat_bucket(int64_t v) {
  if (v <= 0) return 0u;
  return v >= 5 ? 10u : (uint32_t)(2 * v);
}

// kPass 0: each entry's life as event positions (delta[first] += 1, delta[gone] -= 1; no
// other effect) for the capacity check.  kPass 1: the join's effects -- histograms,
// no_response, the carry-out -- unless the capacity bound (the host's sequential replay).
// An entry leaves at the reply that deletes it, or just before the first record event
// whose clock passes its expiry (the cleaner evicts it then).
template <int kPass>
__global__ __launch_bounds__(kLatThreads) void lat_walk_kernel(LatArgs a, uint32_t enabled) {
  const uint64_t n = a.state[kLatEvents];
  if (kPass == 1 && *a.max_live > (int64_t)a.limit) return;
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long h = a.hash_out[i];
  if (i > 0 && a.hash_out[i - 1] == h) return;  // not a segment start
  uint64_t j = i + 1;
  while (j < n && a.hash_out[j] == h) ++j;
  const unsigned long long clk_end = a.state[kLatClockEnd];
  const uint64_t pend = a.state[kLatPending];
  unsigned long long *st = a.state;
  // first record event (positions >= pend, clocks non-decreasing) whose clock passes `exp`
  auto gone_at = [&](unsigned long long exp) {
    uint64_t lo = pend, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (a.ev[mid].clock > exp) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  };
  auto life = [&](uint64_t first, uint64_t gone) {  // kPass 0
    atomicAdd(&a.delta[first], 1);
    atomicAdd(&a.delta[gone], -1);
  };
  // one pass per distinct exact key of the segment (a 64-bit hash collision is the only
  // way a segment holds two); events of a key in record order (stable sort)
  for (uint64_t p = i; p < j; ++p) {
    const LatEvent ep = a.ev[a.idx_out[p]];
    bool seen = false;
    for (uint64_t q = i; q < p && !seen; ++q) {
      const LatEvent eq = a.ev[a.idx_out[q]];
      seen = eq.k0 == ep.k0 && eq.k1 == ep.k1;
    }
    if (seen) continue;
    bool live = false, syn = false;
    unsigned long long expires = 0;
    uint64_t first = 0, touch = 0;
    uint32_t nanos = 0;
    for (uint64_t q = p; q < j; ++q) {
      const uint64_t pos = a.idx_out[q];
      const LatEvent e = a.ev[pos];
      if (e.k0 != ep.k0 || e.k1 != ep.k1) continue;
      const uint32_t role = e.bits & 3u;
      if (role == kRoleCarry) {  // pending from an earlier batch: first in order
        live = true;
        expires = e.clock;
        nanos = e.nanos;
        syn = (e.bits >> 2) & 1u;
        first = pos;
        touch = e.seq;
        continue;
      }
      if (live && e.clock > expires) {  // the cleaner evicted it before this record
        live = false;
        if (kPass == 0) life(first, gone_at(expires));
        else if (enabled & 4u) atomicAdd(&st[kLatNoResponse], 1ULL);
      }
      if (role == kRoleReq) {
        if (!live) {  // Set
          live = true;
          nanos = e.nanos;
          syn = (e.bits >> 2) & 1u;
          first = pos;
        }
        expires = e.clock + kLatTtlNs;  // Set, or the Get hit's touch
        touch = e.seq;
      } else if (live) {  // reply: latency of the first reply, then Delete
        if (kPass == 0) {
          life(first, pos);
        } else {
          const int64_t d = (int64_t)e.nanos - (int64_t)nanos;
          const int64_t ad = d < 0 ? -d : d;
          const int64_t lat = (d < 0 ? -1 : 1) * ((ad + 500000) / 1000000);  // math.Round
          const uint32_t bk = lat_bucket(lat);
          if (enabled & 1u) {
            atomicAdd(&st[kLatHist + bk], 1ULL);
            atomicAdd(&st[kLatHist + 11], 1ULL);
            atomicAdd(&st[kLatHist + 12], (unsigned long long)lat);
          }
          if ((enabled & 2u) && syn && ((e.bits >> 2) & 1u) && ((e.bits >> 3) & 1u)) {
            atomicAdd(&st[kLatHandshake + bk], 1ULL);
            atomicAdd(&st[kLatHandshake + 11], 1ULL);
            atomicAdd(&st[kLatHandshake + 12], (unsigned long long)lat);
          }
        }
        live = false;
      }
    }
    if (!live) continue;
    if (clk_end > expires) {
      if (kPass == 0) life(first, gone_at(expires));
      else if (enabled & 4u) atomicAdd(&st[kLatNoResponse], 1ULL);
    } else if (kPass == 0) {
      atomicAdd(&a.delta[first], 1);
    } else {
      const unsigned long long o = atomicAdd(&st[kLatCarryOut], 1ULL);
      a.carry_out[o] = LatEvent{ep.k0, ep.k1, expires, touch, nanos, kRoleCarry | (syn ? 4u : 0u)};
    }
  }
}

__global__ void lat_finish_kernel(unsigned long long *st, const int32_t *max_live, uint64_t limit,
                                  uint32_t guard) {
  // guard: a capacity-bound batch is finished after its host replay (lat_resolve)
  if (guard && max_live && *max_live > (int64_t)limit) return;
  st[kLatSeqBase] += st[kLatEvents] - st[kLatPending];
  st[kLatClock] = st[kLatClockEnd];
  st[kLatPending] = st[kLatCarryOut];
  const unsigned long long peak = max_live ? (unsigned long long)min((int64_t)*max_live, (int64_t)limit) : 0ULL;
  st[kLatPeakLive] = max(st[kLatPeakLive], max(peak, st[kLatPending]));
}

__global__ void lat_order_init_kernel(const LatEvent *carry, size_t n, unsigned long long *keys, uint32_t *vals) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    keys[e] = carry[e].seq;
    vals[e] = (uint32_t)e;
  }
}

// ---- host side ----------------------------------------------------------------------
hipError_t launch_latency_front(const LatArgs &a, hipStream_t st) {
  const uint32_t wg = (a.blocks + kLatThreads / 64 - 1) / (kLatThreads / 64);  // a.blocks = units (waves)
  hipLaunchKernelGGL(lat_count_kernel, dim3(wg), dim3(kLatThreads), 0, st, a);
  hipLaunchKernelGGL(lat_scan_kernel, dim3(1), dim3(1024), 0, st, a);
  hipLaunchKernelGGL(lat_emit_kernel, dim3(wg), dim3(kLatThreads), 0, st, a);
  hipLaunchKernelGGL(lat_carry_kernel, dim3(64), dim3(256), 0, st, a);
  return hipGetLastError();
}

// Temporary storage for the pass's rocprim calls over n events: the hash sort, the
// carried entries' LRU sort, the live-count scan and its maximum (one buffer, the largest).
hipError_t latency_sort_bytes(size_t n, size_t *bytes) {
  size_t a = 0, b = 0, c = 0;
  hipError_t e = rocprim::radix_sort_pairs(nullptr, a, (const unsigned long long *)nullptr,
                                           (unsigned long long *)nullptr, (const uint32_t *)nullptr,
                                           (uint32_t *)nullptr, n, 0, 64, (hipStream_t)0);
  if (e != hipSuccess) return e;
  if ((e = rocprim::inclusive_scan(nullptr, b, (const int32_t *)nullptr, (int32_t *)nullptr, n + 1,
                                   rocprim::plus<int32_t>(), (hipStream_t)0)) != hipSuccess)
    return e;
  if ((e = rocprim::reduce(nullptr, c, (const int32_t *)nullptr, (int32_t *)nullptr, (int32_t)0, n + 1,
                           rocprim::maximum<int32_t>(), (hipStream_t)0)) != hipSuccess)
    return e;
  *bytes = std::max(a, std::max(b, c));
  return hipSuccess;
}

hipError_t latency_carry_order(const LatEvent *carry, size_t n, unsigned long long *keys, uint32_t *vals,
                               void *tmp, size_t tmp_bytes, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(lat_order_init_kernel, dim3((uint32_t)std::min<size_t>(1024, (n + 255) / 256)), dim3(256),
                     0, st, carry, n, keys, vals);
  size_t tb = tmp_bytes;
  return rocprim::radix_sort_pairs(tmp, tb, keys, keys + n, vals, vals + n, n, 0, 64, st);
}

hipError_t launch_latency_check(const LatArgs &a, size_t n_events, void *tmp, size_t tmp_bytes,
                                uint32_t enabled, hipStream_t st) {
  hipError_t e;
  if (n_events) {
    size_t tb = tmp_bytes;
    if ((e = rocprim::radix_sort_pairs(tmp, tb, a.hash_in, a.hash_out, a.idx_in, a.idx_out, n_events, 0, 64,
                                       st)) != hipSuccess)
      return e;
    const dim3 grid((uint32_t)((n_events + kLatThreads - 1) / kLatThreads));
    // capacity check: entry lives as +1 / -1 at event positions, the live count before
    // each event (prefix sums) and its maximum
    if ((e = hipMemsetAsync(a.delta, 0, (n_events + 1) * sizeof(int32_t), st)) != hipSuccess) return e;
    hipLaunchKernelGGL(lat_walk_kernel<0>, grid, dim3(kLatThreads), 0, st, a, enabled);
    tb = tmp_bytes;
    if ((e = rocprim::inclusive_scan(tmp, tb, a.delta, a.live, n_events + 1, rocprim::plus<int32_t>(), st)) !=
        hipSuccess)
      return e;
    tb = tmp_bytes;
    if ((e = rocprim::reduce(tmp, tb, a.live, a.max_live, (int32_t)0, n_events + 1, rocprim::maximum<int32_t>(),
                             st)) != hipSuccess)
      return e;
  }
  return hipGetLastError();
}

hipError_t launch_latency_walk(const LatArgs &a, size_t n_events, uint32_t enabled, hipStream_t st) {
  if (!n_events) return hipSuccess;
  hipLaunchKernelGGL(lat_walk_kernel<1>, dim3((uint32_t)((n_events + kLatThreads - 1) / kLatThreads)),
                     dim3(kLatThreads), 0, st, a, enabled);
  return hipGetLastError();
}

hipError_t launch_latency_finish(const LatArgs &a, size_t n_events, bool guard, hipStream_t st) {
  hipLaunchKernelGGL(lat_finish_kernel, dim3(1), dim3(1), 0, st, a.state, n_events ? a.max_live : nullptr,
                     a.limit, guard ? 1u : 0u);
  return hipGetLastError();
}

}  // namespace gpuagg
