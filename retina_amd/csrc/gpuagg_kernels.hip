// gfx950 kernels of the flow-aggregation engine.
//
// aggregate_kernel fuses, per flow record, what the reference does in three
// goroutines: the enricher's two IP lookups (enricher.go:117-130, cache.go:154-169),
// the metric dispatch (metrics_module.go:282-297) and every enabled metric's
// ProcessFlow label group-by (forward.go:150-224, drops.go:315-395,
// tcpflags.go:68-132, tcpretrans.go:247-298, dns.go:462-540), plus the count-min /
// HyperLogLog sketch updates (new).
//
// Dense local-context counters are privatised per workgroup in LDS when the group
// key space fits (see DenseLds below) and flushed once per workgroup with coalesced
// 64-bit atomics; everything else goes straight to HBM with device-scope atomics.
#include <hip/hip_runtime.h>

#include "gpuagg_internal.h"

namespace gpuagg {

struct DevIpTable {
  const uint64_t *slots;
  uint32_t mask;
};
struct DevDense {
  unsigned long long *cnt;
  unsigned long long *byt;
};
struct DevSparse {
  unsigned long long *k0, *k1, *k2, *cnt, *byt;
  uint32_t mask;
  unsigned long long *dropped;
};
struct DevSketch {
  uint32_t *cms;
  uint32_t depth;
  uint32_t wlog2;
  uint32_t *hll;  // u8 registers viewed as u32 words
  uint32_t p;     // 0 = off
};
struct DevCols {
  const uint32_t *src, *dst, *bytes, *meta, *ports, *dns;
};

struct Lk {
  int32_t slot;  // -1: not a pod (flow.Endpoint stays nil)
  uint32_t api;  // endpoint is the kubernetes-apiserver pseudo pod (types.go:358-368)
};

__device__ __forceinline__ Lk ip_lookup(const DevIpTable &t, uint32_t ip) {
  uint32_t h = ip_hash(ip) & t.mask;
  for (;;) {
    const uint64_t e = t.slots[h];
    if (e == kIpEmpty) return Lk{-1, 0};
    if ((uint32_t)e == ip) return Lk{(int32_t)((e >> 32) & ((1u << kSlotBits) - 1)), (uint32_t)(e >> 53) & 1u};
    h = (h + 1) & t.mask;
  }
}

// Insert-or-add into the sparse table. No lane ever waits for another: a lane that
// meets a slot whose key is still being published moves on, so a key may occupy
// more than one slot; the host sums duplicates when it renders series.
__device__ __forceinline__ void sparse_add(const DevSparse &s, uint64_t k0, uint64_t k1,
                                           uint64_t k2, uint64_t c, uint64_t b) {
  uint32_t h = (uint32_t)key_hash(k0, k1, k2) & s.mask;
  for (uint32_t probe = 0; probe < kSparseMaxProbe; ++probe) {
    const unsigned long long cur = atomicCAS(&s.k0[h], 0ULL, (unsigned long long)k0);
    if (cur == 0ULL) {
      atomicExch(&s.k1[h], (unsigned long long)k1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      atomicExch(&s.k2[h], (unsigned long long)k2);  // publish
      atomicAdd(&s.cnt[h], (unsigned long long)c);
      if (b) atomicAdd(&s.byt[h], (unsigned long long)b);
      return;
    }
    if (cur == k0) {
      const unsigned long long c2 = atomicCAS(&s.k2[h], kKeyPending, kKeyPending);
      if (c2 == k2) {
        const unsigned long long c1 = atomicCAS(&s.k1[h], 0ULL, 0ULL);
        if (c1 == k1) {
          atomicAdd(&s.cnt[h], (unsigned long long)c);
          if (b) atomicAdd(&s.byt[h], (unsigned long long)b);
          return;
        }
      }
    }
    h = (h + 1) & s.mask;
  }
  atomicAdd(s.dropped, 1ULL);
}

// Side tuple of a context (types.go:418-505): only the fields the options read.
struct SideKey {
  uint32_t ip, slot1, port17;
};
__device__ __forceinline__ SideKey side_key(uint32_t opts, uint32_t ip, const Lk &lk,
                                            uint32_t port, uint32_t proto) {
  SideKey k;
  k.ip = (opts & OPT_IP) ? ip : 0u;
  k.slot1 = (opts & OPT_EP) ? (uint32_t)(lk.slot + 1) : 0u;
  k.port17 = ((opts & OPT_PORT) && (proto == 6 || proto == 17)) ? (0x10000u | port) : 0u;
  return k;
}

__device__ __forceinline__ bool family_matches(uint32_t fam, uint32_t verdict, uint32_t proto,
                                               uint32_t dnstype, uint32_t flagmask) {
  switch (fam) {
    case FAM_FWD: return verdict == kVerdictForwarded;
    case FAM_DROP: return verdict == kVerdictDropped;
    case FAM_TCPFLAGS: return verdict == kVerdictForwarded && proto == 6 && flagmask != 0;
    case FAM_RETRANS: return verdict == kVerdictRetrans;
    case FAM_DNS_REQ: return verdict == kVerdictDns && dnstype == kDnsQuery;
    case FAM_DNS_RESP: return verdict == kVerdictDns && dnstype == kDnsResponse;
  }
  return false;
}

__device__ __forceinline__ void dense_add(const DevDense &d, uint64_t idx, uint32_t fam,
                                          uint32_t nbytes) {
  atomicAdd(&d.cnt[idx], 1ULL);
  if (fam <= FAM_DROP && nbytes) atomicAdd(&d.byt[idx], (unsigned long long)nbytes);
}

// One record through every metric group.
__device__ __forceinline__ void apply_groups(const Plan &p, const DevDense &d,
                                             const DevSparse &s, uint32_t sip, uint32_t dip,
                                             uint32_t nbytes, uint32_t meta, uint32_t ports,
                                             uint32_t dns, const Lk &ls, const Lk &ld) {
  const uint32_t proto = meta_proto(meta), verdict = meta_verdict(meta);
  const uint32_t tdir = meta_tdir(meta), reason = meta_reason(meta);
  const uint32_t dnstype = meta_dnstype(meta);
  const uint32_t flagmask = (verdict == kVerdictForwarded && proto == 6)
                                ? flag_label_mask(meta_flags(meta)) : 0u;
  const uint32_t sport = ports & 0xFFFFu, dport = ports >> 16;

  for (int g = 0; g < p.ngroups; ++g) {
    const GroupPlan gp = p.g[g];
    const uint32_t fam = gp.family;
    if (!family_matches(fam, verdict, proto, dnstype, flagmask)) continue;
    const uint64_t addb = (fam <= FAM_DROP) ? nbytes : 0u;

    if (p.local) {
      // getLocalCtxValues (types.go:379-416): src -> egress, dst -> ingress, both
      // skipped when nil or the apiserver pseudo pod; no values when no option is set.
      if (gp.src_opts == 0) continue;
      const bool s_ok = ls.slot >= 0 && !ls.api;
      const bool d_ok = ld.slot >= 0 && !ld.api;
      if (fam == FAM_DNS_REQ || fam == FAM_DNS_RESP) {
        // dns.go:506-540: exactly one update; both sides -> pick by TrafficDirection.
        int side;
        if (s_ok && d_ok) side = (tdir == 1) ? 0 : 1;
        else if (d_ok) side = 0;
        else if (s_ok) side = 1;
        else continue;
        const SideKey k = side == 0 ? side_key(gp.src_opts, dip, ld, dport, proto)
                                    : side_key(gp.src_opts, sip, ls, sport, proto);
        sparse_add(s, key0(g, (uint32_t)side, k.slot1, k.ip), key1(k.port17, 0, 0),
                   key2(0, dns), 1, 0);
        continue;
      }
      for (int side = 0; side < 2; ++side) {  // 0 ingress (dst), 1 egress (src)
        const bool ok = side == 0 ? d_ok : s_ok;
        if (!ok) continue;
        const Lk &lk = side == 0 ? ld : ls;
        if (!gp.sparse) {
          const uint64_t key = gp.key_mode ? (uint64_t)lk.slot : 0u;
          const uint64_t row = gp.dense_base + (key * 2 + (uint64_t)side) * gp.nsub;
          if (fam == FAM_TCPFLAGS) {
            for (uint32_t m = flagmask; m; m &= m - 1) dense_add(d, row + __builtin_ctz(m), fam, 0);
          } else {
            dense_add(d, row + (fam == FAM_DROP ? reason : 0u), fam, nbytes);
          }
        } else {
          const SideKey k = side == 0 ? side_key(gp.src_opts, dip, ld, dport, proto)
                                      : side_key(gp.src_opts, sip, ls, sport, proto);
          if (fam == FAM_TCPFLAGS) {
            for (uint32_t m = flagmask; m; m &= m - 1) {
              const uint32_t sub = ((uint32_t)__builtin_ctz(m) << 3) | (uint32_t)side;
              sparse_add(s, key0(g, sub, k.slot1, k.ip), key1(k.port17, 0, 0), 0, 1, 0);
            }
          } else {
            const uint32_t sub = ((fam == FAM_DROP ? reason : 0u) << 3) | (uint32_t)side;
            sparse_add(s, key0(g, sub, k.slot1, k.ip), key1(k.port17, 0, 0), 0, 1, addb);
          }
        }
      }
    } else {
      // Remote context: one tuple [prefix labels] + source values + destination values.
      const SideKey ks = side_key(gp.src_opts, sip, ls, sport, proto);
      const SideKey kd = side_key(gp.dst_opts, dip, ld, dport, proto);
      const uint64_t k1 = key1(ks.port17, kd.port17, kd.slot1);
      if (fam == FAM_TCPFLAGS) {
        for (uint32_t m = flagmask; m; m &= m - 1) {
          const uint32_t sub = (uint32_t)__builtin_ctz(m) << 3;
          sparse_add(s, key0(g, sub, ks.slot1, ks.ip), k1, key2(kd.ip, 0), 1, 0);
        }
      } else {
        uint32_t sub = 0, dnsv = 0;
        if (fam == FAM_FWD || fam == FAM_RETRANS) sub = tdir << 1;
        else if (fam == FAM_DROP) sub = (reason << 3) | (tdir << 1);
        else dnsv = dns;
        sparse_add(s, key0(g, sub, ks.slot1, ks.ip), k1, key2(kd.ip, dnsv), 1, addb);
      }
    }
  }
}

__device__ __forceinline__ void sketch_update(const DevSketch &sk, uint32_t sip, uint32_t dip,
                                              uint32_t ports, uint32_t proto, const Lk &ls) {
  if (sk.depth) {
    const uint64_t base = cms_base(sip, dip, ports, proto);
    const uint32_t wmask = (1u << sk.wlog2) - 1u;
    for (uint32_t r = 0; r < sk.depth; ++r)
      atomicAdd(&sk.cms[((size_t)r << sk.wlog2) + cms_col(base, r, wmask)], 1u);
  }
  if (sk.p && ls.slot >= 0) {
    const uint64_t h = hll_hash(dip);
    const uint32_t idx = (uint32_t)(h >> (64 - sk.p));
    const uint64_t w = (h << sk.p) | (1ULL << (sk.p - 1));
    const uint32_t rho = (uint32_t)__builtin_clzll(w) + 1u;
    const size_t byte = ((size_t)ls.slot << sk.p) + idx;
    uint32_t *word = sk.hll + (byte >> 2);
    const uint32_t sh = (uint32_t)(byte & 3) * 8u;
    uint32_t old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (((old >> sh) & 0xFFu) < rho) {
      const uint32_t nw = (old & ~(0xFFu << sh)) | (rho << sh);
      const uint32_t prev = atomicCAS(word, old, nw);
      if (prev == old) break;
      old = prev;
    }
  }
}

template <bool kSketch>
__global__ __launch_bounds__(256) void aggregate_kernel(DevCols c, uint32_t n, DevIpTable t,
                                                        Plan p, DevDense d, DevSparse s,
                                                        DevSketch sk) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t sip = c.src[i], dip = c.dst[i], nbytes = c.bytes[i], meta = c.meta[i];
    const uint32_t ports = (p.need_ports || kSketch) ? c.ports[i] : 0u;
    const uint32_t dns = p.need_dns ? c.dns[i] : 0u;
    const Lk ls = ip_lookup(t, sip);
    const Lk ld = ip_lookup(t, dip);
    apply_groups(p, d, s, sip, dip, nbytes, meta, ports, dns, ls, ld);
    if (kSketch) sketch_update(sk, sip, dip, ports, meta_proto(meta), ls);
  }
}

__global__ void sparse_init_kernel(unsigned long long *k2, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    k2[i] = kKeyPending;
}

__global__ void sparse_export_kernel(DevSparse s, size_t cap_slots, unsigned long long *out,
                                     size_t out_cap, unsigned long long *counter) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < cap_slots;
       i += (size_t)gridDim.x * blockDim.x) {
    const unsigned long long k0 = s.k0[i];
    if (!k0) continue;
    const unsigned long long pos = atomicAdd(counter, 1ULL);
    if (pos >= out_cap) continue;
    unsigned long long *o = out + pos * kSparseEntryWords;
    o[0] = k0;
    o[1] = s.k1[i];
    o[2] = s.k2[i];
    o[3] = s.cnt[i];
    o[4] = s.byt[i];
  }
}

__global__ void sparse_import_kernel(DevSparse s, const unsigned long long *in, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const unsigned long long *e = in + i * kSparseEntryWords;
    sparse_add(s, e[0], e[1], e[2], e[3], e[4]);
  }
}

}  // namespace gpuagg

// ---- launch wrappers called by the host runtime ---------------------------------------
#include "gpuagg_launch.h"

namespace gpuagg {

static DevSparse dev_sparse(const SparseView &v) {
  return DevSparse{(unsigned long long *)v.k0, (unsigned long long *)v.k1,
                   (unsigned long long *)v.k2, (unsigned long long *)v.cnt,
                   (unsigned long long *)v.byt, v.mask, (unsigned long long *)v.dropped};
}

hipError_t launch_aggregate(const LaunchArgs &a, hipStream_t st) {
  DevCols c{a.cols.src_ip, a.cols.dst_ip, a.cols.bytes, a.cols.meta, a.cols.ports, a.cols.dns_id};
  DevIpTable t{a.ip_slots, a.ip_mask};
  DevDense d{(unsigned long long *)a.dense_cnt, (unsigned long long *)a.dense_byt};
  DevSparse s = dev_sparse(a.sparse);
  DevSketch sk{a.cms, a.cms_depth, a.cms_wlog2, (uint32_t *)a.hll, a.hll_p};
  const bool sketch = a.cms_depth || a.hll_p;
  uint32_t blocks = (uint32_t)((a.n + 255) / 256);
  if (blocks > a.max_blocks) blocks = a.max_blocks;
  if (blocks == 0) return hipSuccess;
  if (sketch)
    hipLaunchKernelGGL(aggregate_kernel<true>, dim3(blocks), dim3(256), 0, st, c, (uint32_t)a.n, t,
                       a.plan, d, s, sk);
  else
    hipLaunchKernelGGL(aggregate_kernel<false>, dim3(blocks), dim3(256), 0, st, c, (uint32_t)a.n,
                       t, a.plan, d, s, sk);
  return hipGetLastError();
}

hipError_t launch_sparse_init(const SparseView &v, size_t slots, hipStream_t st) {
  hipLaunchKernelGGL(sparse_init_kernel, dim3(2048), dim3(256), 0, st,
                     (unsigned long long *)v.k2, slots);
  return hipGetLastError();
}

hipError_t launch_sparse_export(const SparseView &v, size_t slots, uint64_t *out, size_t out_cap,
                                uint64_t *counter, hipStream_t st) {
  hipLaunchKernelGGL(sparse_export_kernel, dim3(2048), dim3(256), 0, st, dev_sparse(v), slots,
                     (unsigned long long *)out, out_cap, (unsigned long long *)counter);
  return hipGetLastError();
}

hipError_t launch_sparse_import(const SparseView &v, const uint64_t *in, size_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  uint32_t blocks = (uint32_t)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(sparse_import_kernel, dim3(blocks), dim3(256), 0, st, dev_sparse(v),
                     (const unsigned long long *)in, n);
  return hipGetLastError();
}

}  // namespace gpuagg
