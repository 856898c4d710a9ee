// gfx950 kernels of the flow-aggregation engine.
//
// aggregate_kernel fuses, per flow record, what the reference does in three
// goroutines: the enricher's two IP lookups (enricher.go:117-130, cache.go:154-169),
// the metric dispatch (metrics_module.go:282-297) and every enabled metric's
// ProcessFlow label group-by (forward.go:150-224, drops.go:315-395,
// tcpflags.go:68-132, tcpretrans.go:247-298, dns.go:462-540), plus the count-min /
// HyperLogLog sketch updates (new).
//
// Memory plan:
//  * records stream from HBM once, 16 B per lane per column (dwordx4) when aligned;
//  * the IP table (<= a few MB) stays in each XCD's L2;
//  * dense counters [0, L) are privatised per workgroup in LDS (one 1024-thread
//    workgroup per CU, 160 KB) as packed count<<40|bytes words and flushed once per
//    workgroup with coalesced 64-bit atomics;
//  * dense counters >= L are appended to a per-workgroup spill list (no global
//    atomics, no global counter) and folded by spill_window_kernel, which holds one
//    160 KB window of them in LDS per workgroup;
//  * sparse (remote-context / ip / port / DNS) keys go to an HBM hash table.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "gpuagg_internal.h"
#include "gpuagg_launch.h"

namespace gpuagg {

struct DevIpTable {
  const uint64_t *slots;  // buckets of 2 entries (16 bytes)
  uint32_t mask;          // bucket mask
  uint32_t seed;
  const uint16_t *pre;    // radix table (kRadix*), or null
  const uint32_t *blk;
  // radix table with at most kRadixSmall /16 prefixes (the usual pod CIDRs): the
  // prefixes themselves, block j's in 16 bits of rp[j / 2]; the block of an address is
  // found by compares instead of a load from `pre` (one dependent gather per lookup
  // instead of two).  rpn = 0: use `pre`.
  uint32_t rpn;
  uint32_t rp[kRadixSmall / 2];
};

// Radix block of ip: compares against the few prefixes, else the `pre` table.
__device__ __forceinline__ uint32_t radix_block(const DevIpTable &t, uint32_t ip) {
  if (!t.rpn) return t.pre[ip & 0xFFFFu];
  const uint32_t lo = ip & 0xFFFFu;
  uint32_t b = kRadixNoBlock;
#pragma unroll
  for (uint32_t j = 0; j < kRadixSmall; ++j)
    b = (j < t.rpn && lo == ((t.rp[j >> 1] >> ((j & 1u) * 16u)) & 0xFFFFu)) ? j : b;
  return b;
}
struct DevDense {
  unsigned long long *cnt;
  unsigned long long *byt;
};
struct DevSparse {
  unsigned long long *k0, *k1, *k2, *cnt, *byt;
  uint32_t mask;
  unsigned long long *dropped;
  uint32_t compact;  // 64-bit keys (see sparse_add_compact), 2 words per slot at k0
  uint32_t seg_log2; // compact: probes stay in the key's 2^seg_log2-slot segment
  // compact keys bucketed per segment (aggregate_kernel sets this workgroup's lists and
  // the LDS fill counters; null: sparse_insert adds in place)
  unsigned long long *lists;
  uint32_t *lctr;
  uint32_t lcap;
  // per-workgroup LDS cache of hot group-by keys (aggregate_kernel)
  struct HotKey *hot;
  uint32_t hot_n;  // entries, a power of two (0: no cache)
  // doorkeeper bitmap (LDS, 2^door_log2 bits): a wide key may claim a cache entry only
  // when its bit was already set, i.e. (up to collisions) on its second sighting in the
  // workgroup, so the keys seen once -- the long tail -- do not take the entries
  uint32_t *door;
  uint32_t door_log2;  // 0: no doorkeeper
  // wide keys whose port and DNS fields are zero for every group of the plan (no port
  // option, no DNS family), with GPUAGG_FLAG_NARROW_ENTRIES: list entries drop the zero
  // words (list_entry_words)
  uint32_t narrow;
};

// One cached key: tag 0 free, 1 being claimed, 2 published (key words final).
struct HotKey {
  unsigned long long tag, k0, k1, k2, cnt, byt;
};
static_assert(sizeof(HotKey) == kHotKeyBytes, "LDS sizing in gpuagg_runtime.cpp");

// Candidate entries per key.  Entries are never evicted, so a hot key whose candidates are
// all taken by the time it first comes misses for the rest of the launch and appends every
// update: with two, C4-remote's workgroups each lost a few top-100 flows that way and some
// list overflowed in every launch, so every launch folded (a third way: -2.5 % appends,
// fullest list ~2681 -> ~440 in a 4-workgroup simulation of the bench stream)
constexpr uint32_t kHotWays = 3;
// Adds (c, b) to key (k0, k1, k2) (hash h) in this workgroup's LDS hot-key cache if the
// key is there or a free entry can be claimed (kHotWays candidate entries); false: the caller
// adds to the lists / HBM table.  No lane ever waits: an entry being claimed by another
// lane is skipped.  Under skew (C4's Zipf flows) the hot keys then cost LDS atomics
// instead of memory-side atomics serialised on one table slot; the cache is added to the
// table once per workgroup at the end.  Who may claim is the caller's policy (a key seen
// more than once in the wave, or a key the doorkeeper bitmap has seen before).
__device__ __forceinline__ bool hot_add(const DevSparse &s, uint32_t h, uint64_t k0, uint64_t k1, uint64_t k2,
                                        uint64_t c, uint64_t b, bool may_claim) {
#pragma unroll
  for (uint32_t q = 0; q < kHotWays; ++q) {
    HotKey *e = &s.hot[(h + q * 0x9E37u) & (s.hot_n - 1u)];
    unsigned long long t = __hip_atomic_load(&e->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (t == 0ULL) {
      if (!may_claim) continue;
      t = atomicCAS(&e->tag, 0ULL, 1ULL);
      if (t == 0ULL) {  // claimed: write the key and the first update, then publish
        e->k0 = k0;
        e->k1 = k1;
        e->k2 = k2;
        e->cnt = c;
        e->byt = b;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __hip_atomic_store(&e->tag, 2ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return true;
      }
    }
    if (t == 2ULL && e->k0 == k0 && e->k1 == k1 && e->k2 == k2) {
      atomicAdd(&e->cnt, (unsigned long long)c);
      if (b) atomicAdd(&e->byt, (unsigned long long)b);
      return true;
    }
  }
  return false;
}
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

struct KArgs {
  DevCols c;
  uint64_t n;
  uint64_t chunk;  // records per workgroup (multiple of 4)
  DevIpTable t;
  DevDense d;
  DevSparse s;
  DevSketch sk;
  uint32_t lds_bins;  // L: dense bins privatised in LDS (u64 words; tier-1: u32 words)
  // spill lists: per workgroup, one list per fold window of 2^win_shift bins
  // starting at dense bin `spill_lo`; list (b, w) at spill + (b*nwin + w)*spill_cap;
  // entries u32 = bin offset in the window | bytes << win_shift (DenseSink::entry)
  uint32_t spill_cap;
  uint32_t nwin, win_shift, spill_lo;
  uint32_t *spill;  // or null: bins >= lds_bins use global atomics
  uint32_t *spill_count;      // [gridDim.x * nwin]
  // tier-1: LDS image of the IP table
  const uint8_t *ipl;
  uint32_t ipl_nb, ipl_seed, ipl_bytes;
  uint32_t ipl_npfx, ipl_pfx[kIprMaxPfx];  // radix image (dense_lds_kernel kIp 1 / 2)
  uint32_t ipl_dr[kIprMaxPfx];             // dense radix descriptors (kIp 2)
  uint32_t *stage_a;  // tier-1 staged flush: [gridDim.x][stage_a_stride] u32, or null
  uint32_t stage_a_stride;
  uint32_t stage_accum;  // tier-1: bins start from this workgroup's staged copy (deferred reduce)
  // compact group-by keys bucketed per table segment (generic kernel), or null
  unsigned long long *sp_lists;
  uint32_t *sp_counts;
  uint32_t sp_nwin, sp_cap;
  // deferred folds: the lists already hold earlier launches' entries, so this launch's
  // LDS fill counters start from spill_count / sp_counts instead of 0
  uint32_t accum;
  uint32_t hot_n;  // LDS hot-key cache entries of aggregate_kernel (0: none)
  uint32_t door_log2;  // doorkeeper bits of the hot-key cache (0: every key may claim)
  uint32_t row_masks;  // spilled tcpflags rows 8-aligned in their windows: one row-mask entry
  uint32_t *fold_flag;  // wide lists: fullest list of this launch -> fold_flag[fold_parity]
  uint32_t fold_parity;
  Plan p;
};

// This workgroup's fill counter of list w at launch start (deferred folds append after
// the entries earlier launches left).
__device__ __forceinline__ uint32_t spill_ctr0(const KArgs &a, uint32_t w) {
  if (!a.accum) return 0u;
  const uint32_t c = a.spill_count[blockIdx.x * a.nwin + w];
  return c < a.spill_cap ? c : a.spill_cap;
}

struct Lk {
  int32_t slot;  // -1: not a pod (flow.Endpoint stays nil)
  uint32_t api;  // endpoint is the kubernetes-apiserver pseudo pod (types.go:358-368)
};

__device__ __forceinline__ Lk lk_from(uint64_t e) {
  if (e == kIpEmpty) return Lk{-1, 0};
  return Lk{(int32_t)((e >> 32) & ((1u << kSlotBits) - 1)), (uint32_t)(e >> 53) & 1u};
}

// Bucketized cuckoo lookup (host builder: gpuagg_set_endpoints): one 16-byte load of
// the first bucket; the second bucket is read only when the first is full and holds
// neither entry (~15 % of lookups at the 40 % build load).  An EMPTY entry never matches
// a real key because the host refuses 255.255.255.255 as a pod IP.
__device__ __forceinline__ ulonglong2 ip_bucket(const DevIpTable &t, uint32_t b) {
  return ((const ulonglong2 *)t.slots)[b];
}
__device__ __forceinline__ bool ip_need2(uint32_t ip, const ulonglong2 &e) {
  return (uint32_t)e.x != ip && (uint32_t)e.y != ip && e.x != kIpEmpty && e.y != kIpEmpty;
}
__device__ __forceinline__ Lk ip_pick(uint32_t ip, const ulonglong2 &e1, const ulonglong2 &e2) {
  const uint64_t e = (uint32_t)e1.x == ip ? e1.x : (uint32_t)e1.y == ip ? e1.y
                   : (uint32_t)e2.x == ip ? e2.x : (uint32_t)e2.y == ip ? e2.y : kIpEmpty;
  return lk_from(e);
}

__device__ __forceinline__ Lk radix_pick(uint32_t e) {
  return e == kRadixEmpty ? Lk{-1, 0} : Lk{(int32_t)(e & ((1u << kSlotBits) - 1)), e >> 31};
}
__device__ __forceinline__ uint32_t radix_entry(const DevIpTable &t, uint32_t ip, uint32_t b) {
  return b == kRadixNoBlock ? kRadixEmpty : t.blk[(b << 16) | (ip >> 16)];
}

__device__ __forceinline__ Lk ip_lookup(const DevIpTable &t, uint32_t ip) {
  if (t.pre) return radix_pick(radix_entry(t, ip, radix_block(t, ip)));
  const ulonglong2 e1 = ip_bucket(t, ip_h1(ip, t.seed) & t.mask);
  const ulonglong2 e2 = ip_need2(ip, e1) ? ip_bucket(t, ip_h2(ip, t.seed) & t.mask)
                                         : make_ulonglong2(kIpEmpty, kIpEmpty);
  return ip_pick(ip, e1, e2);
}

// Compact table (plans whose every sparse key fits 64 bits: local context whose only
// sparse groups are DNS -- k1 == 0 and k2 = dns id, so key = k0 | dns id): one 16-byte
// slot (key, count) per entry; the claiming CAS publishes the whole key, so an insert is
// one CAS and one add and a key never occupies two slots.
// Linear probing wraps inside the key's segment of 2^seg_log2 slots, so one segment
// (128 KiB) can be folded in LDS (sparse_fold_kernel) with the same probe sequence.
__device__ __forceinline__ uint32_t compact_home(const DevSparse &s, uint64_t key) {
  return (uint32_t)fmix64(key ^ 0x243F6A8885A308D3ULL) & s.mask;
}
__device__ __forceinline__ void sparse_add_compact(const DevSparse &s, uint64_t key, uint64_t c) {
  const uint32_t h = compact_home(s, key), smask = (1u << s.seg_log2) - 1u, seg = h & ~smask;
  for (uint32_t probe = 0; probe <= smask; ++probe) {
    unsigned long long *slot = s.k0 + 2ull * (seg | ((h + probe) & smask));
    const unsigned long long cur = atomicCAS(&slot[0], 0ULL, (unsigned long long)key);
    if (cur == 0ULL || cur == key) {
      atomicAdd(&slot[1], (unsigned long long)c);
      return;
    }
  }
  atomicAdd(s.dropped, 1ULL);
}

// The compact plan's aggregation side: a key goes to its table segment's list (LDS fill
// counter, one 8-byte store); a full list adds in place.  Only the fields this needs, so
// kernels that use it keep few scalar registers live.
struct CompactLists {
  unsigned long long *lists;  // this workgroup's [nseg][lcap] keys
  uint32_t *lctr;             // LDS fill counters
  uint32_t lcap;
  unsigned long long *k0, *dropped;
  uint32_t mask, seg_log2;
  __device__ __forceinline__ void insert(uint64_t key) const {
    const uint32_t h = (uint32_t)fmix64(key ^ 0x243F6A8885A308D3ULL) & mask;  // compact_home
    const uint32_t w = h >> seg_log2;
    const uint32_t pos = atomicAdd(&lctr[w], 1u);
    if (pos < lcap) {
      lists[(size_t)w * lcap + pos] = key;
      return;
    }
    const uint32_t smask = (1u << seg_log2) - 1u, seg = h & ~smask;  // full list: in place (exact)
    for (uint32_t probe = 0; probe <= smask; ++probe) {
      unsigned long long *slot = k0 + 2ull * (seg | ((h + probe) & smask));
      const unsigned long long cur = atomicCAS(&slot[0], 0ULL, (unsigned long long)key);
      if (cur == 0ULL || cur == key) {
        atomicAdd(&slot[1], 1ULL);
        return;
      }
    }
    atomicAdd(dropped, 1ULL);
  }
};

// Insert-or-add into the sparse table. No lane ever waits for another: a lane that
// meets a slot whose key is still being published moves on, so a key may occupy
// more than one slot; the host sums duplicates when it renders series.
__device__ __forceinline__ void sparse_add(const DevSparse &s, uint64_t k0, uint64_t k1,
                                           uint64_t k2, uint64_t c, uint64_t b) {
  if (s.compact) {
    sparse_add_compact(s, k0 | (k2 & 0xFFFFFFFFULL), c);
    return;
  }
  // probing wraps inside the key's segment (the unit sparse_fold_wide_kernel folds)
  const uint32_t h0 = (uint32_t)key_hash(k0, k1, k2) & s.mask, smask = (1u << s.seg_log2) - 1u;
  const uint32_t seg = h0 & ~smask, nprobe = smask < kSparseMaxProbe ? smask + 1u : kSparseMaxProbe;
  for (uint32_t probe = 0; probe < nprobe; ++probe) {
    const uint32_t h = seg | ((h0 + probe) & smask);
    const size_t o = (size_t)h * kSparseSlotWords;  // slot h (k1 = k0 + 1, ...)
    const unsigned long long cur = atomicCAS(&s.k0[o], 0ULL, (unsigned long long)k0);
    if (cur == 0ULL) {
      atomicExch(&s.k1[o], (unsigned long long)k1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      atomicExch(&s.k2[o], (unsigned long long)k2);  // publish
      atomicAdd(&s.cnt[o], (unsigned long long)c);
      if (b) atomicAdd(&s.byt[o], (unsigned long long)b);
      return;
    }
    if (cur == k0) {
      const unsigned long long c2 = atomicCAS(&s.k2[o], kKeyPending, kKeyPending);
      if (c2 == k2) {
        const unsigned long long c1 = atomicCAS(&s.k1[o], 0ULL, 0ULL);
        if (c1 == k1) {
          atomicAdd(&s.cnt[o], (unsigned long long)c);
          if (b) atomicAdd(&s.byt[o], (unsigned long long)b);
          return;
        }
      }
    }
  }
  atomicAdd(s.dropped, c);
}

// words per segment-list entry: compact key 1, wide 4, narrow wide 3
__device__ __forceinline__ uint32_t list_entry_words(const DevSparse &s) {
  return s.compact ? 1u : (s.narrow ? kWideNarrowWords : kWideEntryWords);
}

// Wide keys (192 bits) through per-segment lists: the update is appended to this
// workgroup's list for the key's table segment (LDS fill counter, one 32-byte store) and
// sparse_fold_wide_kernel later adds every list into its segment in LDS -- instead of a
// memory-side CAS + two reads + two adds per cold key.  A full list, or a count / byte
// sum too wide for the entry, goes to the table directly (exact).  kh = key_hash(k0, k1, k2).
__device__ __forceinline__ void wide_append(const DevSparse &s, uint64_t kh, uint64_t k0, uint64_t k1, uint64_t k2,
                                            uint64_t c, uint64_t b) {
  if (c < (1ULL << (kWideHomeShift - kWideCountShift)) && b < (1ULL << kWideCountShift)) {
    const uint32_t w = ((uint32_t)kh & s.mask) >> s.seg_log2;
    const uint32_t pos = atomicAdd(&s.lctr[w], 1u);
    if (pos < s.lcap) {
      const uint64_t home = (uint64_t)((uint32_t)kh & ((1u << s.seg_log2) - 1u));
      const uint64_t m = (home << kWideHomeShift) | (c << kWideCountShift) | b;
      if (s.narrow) {
        unsigned long long *e = s.lists + ((size_t)w * s.lcap + pos) * kWideNarrowWords;
        e[0] = k0;
        e[1] = wide_pack12(k1, k2);
        e[2] = m;
        return;
      }
      ulonglong2 *e = (ulonglong2 *)(s.lists + ((size_t)w * s.lcap + pos) * kWideEntryWords);
      e[0] = make_ulonglong2(k0, k1);
      e[1] = make_ulonglong2(k2, m);
      return;
    }
  }
  sparse_add(s, k0, k1, k2, c, b);
}

// Exact add of one (count 1, bytes nb) update into a packed u64 LDS word
// (count:20 | bytes:44) when a workgroup may exceed the field widths: the lane whose
// add carries out of the bytes field or wraps the count field books the difference
// into the global counters (rare).  Sum over all adds is exact.
__device__ __forceinline__ void lds_add64_exact(unsigned long long *w, uint32_t gbin, uint32_t nb,
                                                const DevDense &d) {
  const uint32_t b = nb < kLdsByteLimit ? nb : 0u;
  const unsigned long long old = atomicAdd(w, kLdsCountOne | b);
  if (nb >= kLdsByteLimit) atomicAdd(&d.byt[gbin], (unsigned long long)nb);
  const unsigned long long carry = ((old & kLdsBytesMask) + b) >> kLdsCountShift;
  const unsigned long long wrap = ((old >> kLdsCountShift) + 1ULL + carry) >> (64 - kLdsCountShift);
  if (carry) {
    atomicAdd(&d.byt[gbin], kLdsCountOne);
    atomicAdd(&d.cnt[gbin], ~0ULL);  // the carry also bumped the count field
  }
  if (wrap) atomicAdd(&d.cnt[gbin], 1ULL << (64 - kLdsCountShift));
}

// Dense counter updates: LDS window, bucketed spill lists, or (fallback) global atomics.
struct DenseSink {
  unsigned long long *lds;  // u64 bins (generic / dense_local kernels)
  uint32_t L;
  unsigned int *ctr;        // per-window spill counters (LDS)
  uint32_t *spill;
  uint32_t spill_cap, win_shift, spill_lo;
  DevDense d;
  uint32_t wbits;           // bits of a window index (nwin <= 2^wbits)

  __device__ __forceinline__ uint32_t window(uint32_t bin) const { return (bin - spill_lo) >> win_shift; }
  // 4-byte entry: the bin's offset in its window and the bytes; bytes that do not fit
  // the field (2^(31 - win_shift): bit 31 marks a row-mask entry, below) are added to the
  // global counter here (rare) and the entry carries 0
  __device__ __forceinline__ uint32_t entry(uint32_t bin, uint32_t nbytes) const {
    const bool fits = (nbytes >> (31u - win_shift)) == 0u;
    if (!fits) atomicAdd(&d.byt[bin], (unsigned long long)nbytes);
    return ((bin - spill_lo) & ((1u << win_shift) - 1u)) | ((fits ? nbytes : 0u) << win_shift);
  }
  // store one reserved spill entry (pos from the window counter); full list -> global
  __device__ __forceinline__ void spill_put(uint32_t bin, uint32_t w, uint32_t pos, uint32_t nbytes) const {
    if (pos < spill_cap) {  // w < 256 and spill_cap < 2^24: 24-bit multiply
      spill[mul_u24(w, spill_cap) + pos] = entry(bin, nbytes);
      return;
    }
    atomicAdd(&d.cnt[bin], 1ULL);
    if (nbytes) atomicAdd(&d.byt[bin], (unsigned long long)nbytes);
  }

  __device__ __forceinline__ void spill_add(uint32_t bin, uint32_t nbytes) const {
    if (spill) {
      const uint32_t w = window(bin);
      const unsigned int pos = atomicAdd(&ctr[w], 1u);
      if (pos < spill_cap) {
        spill[mul_u24(w, spill_cap) + pos] = entry(bin, nbytes);
        return;
      }
    }
    atomicAdd(&d.cnt[bin], 1ULL);
    if (nbytes) atomicAdd(&d.byt[bin], (unsigned long long)nbytes);
  }

  __device__ __forceinline__ void add(uint32_t bin, uint32_t nbytes) const {
    if (bin < L) {
      atomicAdd(&lds[bin], kLdsCountOne | (nbytes < kLdsByteLimit ? nbytes : 0u));
      if (nbytes >= kLdsByteLimit) atomicAdd(&d.byt[bin], (unsigned long long)nbytes);
      return;
    }
    spill_add(bin, nbytes);
  }
};

__device__ __forceinline__ DenseSink make_sink(const KArgs &a, unsigned long long *lds, uint32_t L,
                                               unsigned int *ctr) {
  return DenseSink{lds, L, ctr,
                   a.spill ? a.spill + (size_t)blockIdx.x * a.nwin * a.spill_cap : nullptr,
                   a.spill_cap, a.win_shift, a.spill_lo, a.d,
                   a.nwin > 1 ? 32u - (uint32_t)__builtin_clz(a.nwin - 1) : 0u};
}

__device__ __forceinline__ void spill_counts_out(const KArgs &a, const unsigned int *ctr) {
  if (a.spill)
    for (uint32_t w = threadIdx.x; w < a.nwin; w += blockDim.x)
      a.spill_count[blockIdx.x * a.nwin + w] = ctr[w] < a.spill_cap ? ctr[w] : a.spill_cap;
}

// Positions in the per-window spill lists for the lanes with `ok`, reserved with ONE
// LDS atomic per distinct window of the wave (lanes are grouped by wbits ballots of the
// window bits; the group's lowest lane adds the group size and ds_bpermute hands the
// base to the others).  Per-lane atomics on a few counters serialise in the LDS.
// Must be called by the whole wave.
__device__ __forceinline__ uint32_t wave_reserve(bool ok, uint32_t w, unsigned int *ctr, uint32_t wbits) {
  uint64_t eq = __ballot(ok);
  for (uint32_t b = 0; b < wbits; ++b) {
    const bool bit = (w >> b) & 1u;
    const uint64_t B = __ballot(bit);
    eq &= bit ? B : ~B;
  }
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(eq >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)eq, 0u));
  uint32_t base = 0;
  if (ok && rank == 0) base = atomicAdd(&ctr[w], (uint32_t)__popcll(eq));
  const uint32_t lead = eq ? (uint32_t)__builtin_ctzll(eq) : 0u;
  base = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lead << 2), (int)base);
  return base + rank;
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

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)lane);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {  // converged wave
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// One wide-key update (count 1, bytes b) on the list path: no wave de-duplication (its
// leader loop costs one round per distinct key of a hash-bucket collision -- ~30 rounds
// per insert under C4's Zipf flows, the whole kernel's time).  Lanes with the same key
// meet in the LDS hot-key cache or append separately and are summed by the fold.  A key
// may claim a free cache entry on its second sighting in the workgroup (doorkeeper
// bitmap), so the long tail of keys seen once does not take the entries.
// The cache is searched first and the doorkeeper asked only when one of the key's ways is
// still free: a hit -- or a miss once its ways are taken, i.e. most misses after the first
// records of a launch -- costs no doorkeeper atomic.  (Ways are never freed, so a key
// cannot sit in a later way while an earlier one is free.)
__device__ __forceinline__ void wide_insert(const DevSparse &s, uint64_t k0, uint64_t k1, uint64_t k2, uint64_t b) {
  const uint64_t kh = key_hash(k0, k1, k2);
  if (s.hot_n) {
    const uint32_t h = (uint32_t)kh;
    HotKey *fe = nullptr;
#pragma unroll
    for (uint32_t q = 0; q < kHotWays; ++q) {
      HotKey *e = &s.hot[(h + q * 0x9E37u) & (s.hot_n - 1u)];
      const unsigned long long t = __hip_atomic_load(&e->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (t == 2ULL && e->k0 == k0 && e->k1 == k1 && e->k2 == k2) {
        atomicAdd(&e->cnt, 1ULL);
        if (b) atomicAdd(&e->byt, (unsigned long long)b);
        return;
      }
      if (t == 0ULL && !fe) fe = e;
    }
    if (fe) {
      bool claim = true;
      if (s.door_log2) {
        const uint32_t bit = (uint32_t)(kh >> 40) & ((1u << s.door_log2) - 1u);
        claim = (atomicOr(&s.door[bit >> 5], 1u << (bit & 31u)) >> (bit & 31u)) & 1u;
      }
      if (claim && atomicCAS(&fe->tag, 0ULL, 1ULL) == 0ULL) {  // claimed: key + first update, publish
        fe->k0 = k0;
        fe->k1 = k1;
        fe->k2 = k2;
        fe->cnt = 1ULL;
        fe->byt = b;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __hip_atomic_store(&fe->tag, 2ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return;
      }
    }
  }
  wide_append(s, kh, k0, k1, k2, 1, b);
}

// Wave-level key de-duplication before the global table (BASELINE.json north_star): the
// lanes of a wave inserting the same key merge into the lowest of them, which inserts the
// summed count and bytes once -- a Zipf heavy hitter costs one global CAS/add chain per
// wave instead of one per lane.  Lanes are bucketed by 6 key-hash bits (6 ballots); only
// buckets holding several lanes compare full keys, one leader key per round, so a wave of
// distinct keys pays the ballots and one vote.  Called by the whole wave (converged);
// `valid` is false on lanes with nothing to insert.
__device__ __forceinline__ void sparse_insert(const DevSparse &s, bool valid, uint64_t k0, uint64_t k1,
                                              uint64_t k2, uint64_t b) {
  if (s.lists && s.compact) {  // compact keys: append to the segment's list (LDS fill counter)
    if (!valid) return;
    const uint64_t key = k0 | (k2 & 0xFFFFFFFFULL);
    const uint32_t w = compact_home(s, key) >> s.seg_log2;
    const uint32_t pos = atomicAdd(&s.lctr[w], 1u);
    if (pos < s.lcap) s.lists[(size_t)w * s.lcap + pos] = key;
    else sparse_add_compact(s, key, 1);  // full list: in place (exact)
    return;
  }
  if (s.lists) {
    if (valid) wide_insert(s, k0, k1, k2, b);
    return;
  }
  const uint64_t vm = __ballot(valid);
  if (!vm) return;
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const uint32_t x = (uint32_t)(k0 ^ (k0 >> 29) ^ k1 ^ (k1 >> 31) ^ k2 ^ (k2 >> 27));
  const uint32_t h = (x * 0x9E3779B1u) >> 26;
  uint64_t eq = vm;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const bool bit = (h >> i) & 1u;
    const uint64_t B = __ballot(bit);
    eq &= bit ? B : ~B;
  }
  bool pending = valid && __popcll(eq) > 1;
  bool keep = valid;
  uint64_t c = 1, pm;
  while ((pm = __ballot(pending)) != 0) {
    const uint32_t leader = (uint32_t)__builtin_ctzll(pm);
    const bool same = pending && k0 == readlane64(k0, leader) && k1 == readlane64(k1, leader) &&
                      k2 == readlane64(k2, leader);
    const uint64_t m = __ballot(same);
    const uint64_t bsum = wave_sum64(same ? b : 0ULL);
    if (same) {
      pending = false;
      if (lane == leader) {
        c = (uint64_t)__popcll(m);
        b = bsum;
      } else {
        keep = false;
      }
    }
  }
  // only keys that occur more than once in the wave (the de-dup count) claim a hot-key
  // entry: under skew those are the hot ones; uniform keys (C1) then cost two tag reads
  if (keep && !(s.hot_n && hot_add(s, (uint32_t)key_hash(k0, k1, k2), k0, k1, k2, c, b, c > 1)))
    sparse_add(s, k0, k1, k2, c, b);
}

// One record through every metric group.  Converged: every lane of the wave runs it
// (inactive lanes carry no endpoint and an unmatched verdict), so the sparse inserts can
// de-duplicate keys across the wave (sparse_insert).
__device__ __forceinline__ void apply_groups(const Plan &p, const DenseSink &ds,
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
    const GroupPlan gp = p.g[g];  // plan: wave-uniform
    const uint32_t fam = gp.family;
    const bool hit = family_matches(fam, verdict, proto, dnstype, flagmask);
    const uint32_t addb = (fam <= FAM_DROP) ? nbytes : 0u;

    if (p.local) {
      // getLocalCtxValues (types.go:379-416): src -> egress, dst -> ingress, both
      // skipped when nil or the apiserver pseudo pod; no values when no option is set.
      if (gp.src_opts == 0) continue;
      const bool s_ok = ls.slot >= 0 && !ls.api;
      const bool d_ok = ld.slot >= 0 && !ld.api;
      if (fam == FAM_DNS_REQ || fam == FAM_DNS_RESP) {
        // dns.go:506-540: exactly one update; both sides -> pick by TrafficDirection.
        const int side = (s_ok && d_ok) ? ((tdir == 1) ? 0 : 1) : (d_ok ? 0 : 1);
        const SideKey k = side == 0 ? side_key(gp.src_opts, dip, ld, dport, proto)
                                    : side_key(gp.src_opts, sip, ls, sport, proto);
        sparse_insert(s, hit && (s_ok || d_ok), key0(g, (uint32_t)side, k.slot1, k.ip), key1(k.port17, 0, 0),
                      key2(0, dns), 0);
        continue;
      }
      for (int side = 0; side < 2; ++side) {  // 0 ingress (dst), 1 egress (src)
        const bool ok = hit && (side == 0 ? d_ok : s_ok);
        const Lk &lk = side == 0 ? ld : ls;
        if (!gp.sparse) {
          if (!ok) continue;
          const uint32_t key = gp.key_mode ? (uint32_t)lk.slot : 0u;
          const uint32_t row = (uint32_t)gp.dense_base + (key * 2u + (uint32_t)side) * gp.nsub;
          if (fam == FAM_TCPFLAGS) {
            for (uint32_t m = flagmask; m; m &= m - 1) ds.add(row + __builtin_ctz(m), 0);
          } else {
            ds.add(row + (fam == FAM_DROP ? reason : 0u), addb);
          }
          continue;
        }
        const SideKey k = side == 0 ? side_key(gp.src_opts, dip, ld, dport, proto)
                                    : side_key(gp.src_opts, sip, ls, sport, proto);
        if (fam == FAM_TCPFLAGS) {
          uint32_t m = ok ? flagmask : 0u;
          while (__ballot(m != 0)) {  // converged: trips = most flags of any lane
            const uint32_t sub = (m ? ((uint32_t)__builtin_ctz(m) << 3) : 0u) | (uint32_t)side;
            sparse_insert(s, m != 0, key0(g, sub, k.slot1, k.ip), key1(k.port17, 0, 0), 0, 0);
            m &= m - 1;
          }
        } else {
          const uint32_t sub = ((fam == FAM_DROP ? reason : 0u) << 3) | (uint32_t)side;
          sparse_insert(s, ok, key0(g, sub, k.slot1, k.ip), key1(k.port17, 0, 0), 0, addb);
        }
      }
    } else {
      // Remote context: one tuple [prefix labels] + source values + destination values.
      const SideKey ks = side_key(gp.src_opts, sip, ls, sport, proto);
      const SideKey kd = side_key(gp.dst_opts, dip, ld, dport, proto);
      const uint64_t k1 = key1(ks.port17, kd.port17, kd.slot1);
      if (fam == FAM_TCPFLAGS) {
        uint32_t m = hit ? flagmask : 0u;
        while (__ballot(m != 0)) {
          const uint32_t sub = m ? (uint32_t)__builtin_ctz(m) << 3 : 0u;
          sparse_insert(s, m != 0, key0(g, sub, ks.slot1, ks.ip), k1, key2(kd.ip, 0), 0);
          m &= m - 1;
        }
      } else {
        uint32_t sub = 0, dnsv = 0;
        if (fam == FAM_FWD || fam == FAM_RETRANS) sub = tdir << 1;
        else if (fam == FAM_DROP) sub = (reason << 3) | (tdir << 1);
        else dnsv = dns;
        sparse_insert(s, hit, key0(g, sub, ks.slot1, ks.ip), k1, key2(kd.ip, dnsv), addb);
      }
    }
  }
}

// HLL register max for (source pod slot, dst): register h >> (64 - p), rank
// clz((h << p) | 2^(p-1)) + 1.  The register word is read first and the CAS loop runs
// only when the rank is larger (rare once a pod's registers have warmed up).
__device__ __forceinline__ void hll_update(uint32_t *hll, uint32_t p, int32_t slot, uint32_t dip) {
  const uint64_t h = hll_hash(dip);
  const uint32_t idx = (uint32_t)(h >> (64 - p));
  const uint64_t w = (h << p) | (1ULL << (p - 1));
  const uint32_t rho = (uint32_t)__builtin_clzll(w) + 1u;
  const size_t byte = ((size_t)slot << p) + idx;
  uint32_t *word = hll + (byte >> 2);
  const uint32_t sh = (uint32_t)(byte & 3) * 8u;
  uint32_t old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (((old >> sh) & 0xFFu) < rho) {
    const uint32_t nw = (old & ~(0xFFu << sh)) | (rho << sh);
    const uint32_t prev = atomicCAS(word, old, nw);
    if (prev == old) break;
    old = prev;
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
  if (sk.p && ls.slot >= 0) hll_update(sk.hll, sk.p, ls.slot, dip);
}

// ---- record streaming -------------------------------------------------------------
// Workgroup b owns records [b*chunk, (b+1)*chunk). With kVec every lane takes 4
// consecutive records per step (16-byte loads per column), issues the 16 IP-table
// loads of their 8 addresses back to back, then walks the 4 records in a rolled loop
// (register rotation keeps one copy of the per-record code).  Both loops are
// wave-uniform -- lanes past the end read the last element and pass an inactive record
// (no endpoint, an unmatched verdict) -- so f may use cross-lane operations.
constexpr uint32_t kInactiveMeta = kVerdictUnencodable << 8;
// Record-stream loads: every column element is read once per launch, so they are
// non-temporal -- the stream does not evict the spill lists, IP tables and staged copies
// that the folds read back from L2 (C2 fold 0.043 -> 0.035 ms, C5 kernel 0.208 ->
// 0.200 ms, profiles/round2/r6c*_*).
__device__ __forceinline__ uint4 rec_ld(const uint4 *p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_nontemporal_load((const v4u *)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Workgroup copy of n 16-byte words from global memory into LDS with 4 loads in flight per
// lane before their LDS stores (a plain loop waits on each load: the compiler cannot move a
// load of a generic pointer above the previous iteration's LDS store).
__device__ __forceinline__ void fill_lds_u4(uint4 *dst, const uint4 *src, uint32_t n) {
  uint32_t i = threadIdx.x;
  for (; i + 3 * blockDim.x < n; i += 4 * blockDim.x) {
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = src[i + q * blockDim.x];
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[i + q * blockDim.x] = v[q];
  }
  for (; i < n; i += blockDim.x) dst[i] = src[i];
}

// Probe of the LDS cuckoo image: two 8-byte bucket reads and 4 compares give the index
// of the matching key (or ~0u); the u16 slot id is read separately so all key reads of
// a thread's records can be in flight together.
__device__ __forceinline__ uint32_t ipl_probe_index(const uint32_t *keys, uint32_t nb, uint32_t seed,
                                                    uint32_t ip) {
  uint32_t b1, b2;
  ipl_buckets(ip, seed, nb, b1, b2);
  const uint2 k1 = *(const uint2 *)&keys[b1 * 2], k2 = *(const uint2 *)&keys[b2 * 2];
  uint32_t j = nb * 2;  // sentinel entry: kIplNoSlot
  j = k1.x == ip ? b1 * 2 : j;
  j = k1.y == ip ? b1 * 2 + 1 : j;
  j = k2.x == ip ? b2 * 2 : j;
  j = k2.y == ip ? b2 * 2 + 1 : j;
  return j;
}

// slot id, or kIplNoSlot (not a pod, or the apiserver pseudo pod)
__device__ __forceinline__ uint32_t ipl_slot(const uint16_t *vals, uint32_t j) { return vals[j]; }

// One IP through the tier-1 LDS image: slot or kIplNoSlot (inactive lanes: kIplNoSlot).
// kRadix: the radix image (two dependent u16 reads); else the cuckoo image.
template <int kIp>
struct IplView {
  const uint8_t *smem;
  uint32_t nb, seed, npfx, p0, p1, p2, p3;
  uint32_t d0, d1, d2, d3;  // kIp 2: the dense radix descriptors
  __device__ __forceinline__ uint32_t lookup(uint32_t ip) const {
    if (kIp == 2)
      return ((const uint16_t *)smem)[(iprd_block(ip, p0, p1, p2, p3, d0, d1, d2, d3) << 8) | (ip >> 24)];
    if (kIp == 1) {
      const uint16_t *bidx = (const uint16_t *)smem, *blk = (const uint16_t *)(smem + ipr_blk_offset(npfx));
      return blk[((uint32_t)bidx[ipr_row(ip, p0, p1, p2, p3, npfx)] << 8) | (ip >> 24)];
    }
    return ipl_slot((const uint16_t *)(smem + ipl_vals_offset(nb)), ipl_probe_index((const uint32_t *)smem, nb, seed, ip));
  }
  // the 8 IPs of a step, every read of a level issued before the next level; lookups run
  // for every lane (inactive lanes hold a clamped real record) and the result is masked
  // after: a select on the index made the compiler branch per IP
  __device__ __forceinline__ void lookup8(const uint32_t (&ip)[8], bool act, uint32_t (&sl)[8]) const {
    if (kIp == 2) {  // one LDS read per IP
      const uint16_t *blk = (const uint16_t *)smem;
#pragma unroll
      for (int k = 0; k < 8; ++k) sl[k] = blk[(iprd_block(ip[k], p0, p1, p2, p3, d0, d1, d2, d3) << 8) | (ip[k] >> 24)];
    } else if (kIp == 1) {
      const uint16_t *bidx = (const uint16_t *)smem, *blk = (const uint16_t *)(smem + ipr_blk_offset(npfx));
      uint32_t bi[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) bi[k] = bidx[ipr_row(ip[k], p0, p1, p2, p3, npfx)];
#pragma unroll
      for (int k = 0; k < 8; ++k) sl[k] = blk[(bi[k] << 8) | (ip[k] >> 24)];
    } else {
      const uint32_t *keys = (const uint32_t *)smem;
      const uint16_t *vals = (const uint16_t *)(smem + ipl_vals_offset(nb));
      uint32_t j[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) j[k] = ipl_probe_index(keys, nb, seed, ip[k]);
#pragma unroll
      for (int k = 0; k < 8; ++k) sl[k] = ipl_slot(vals, j[k]);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) sl[k] = act ? sl[k] : kIplNoSlot;
  }
};

// IP lookups of for_each_record: the HBM table, or an LDS image of every pod IP (LdsIp:
// the slot only -- the remote context never reads the apiserver flag)
struct HbmIp {
  static constexpr bool kLds = false;
};
template <int kIp>
struct LdsIp {
  static constexpr bool kLds = true;
  IplView<kIp> iv;
};

struct NoRounds {
  __device__ __forceinline__ void operator()() const {}
};
// kRounds: the vector loop is block-uniform (waves past the end process inactive lanes)
// and calls round_end() after every step, so the caller can flush LDS staging between
// barriers.
template <bool kVec, bool kRounds = false, class F, class RE = NoRounds, class IP = HbmIp>
__device__ __forceinline__ void for_each_record(const KArgs &a, bool need_ports, bool need_dns, F &&f,
                                                RE &&round_end = RE{}, const IP &ipv = IP{}) {
  const bool need_bytes = a.p.need_bytes;  // no forward / drop group: the column is not read
  const uint64_t start = (uint64_t)blockIdx.x * a.chunk;
  const uint64_t end = start + a.chunk < a.n ? start + a.chunk : a.n;
  const uint32_t lane = threadIdx.x & 63u, wave0 = threadIdx.x & ~63u;
  const Lk none{-1, 0};
  uint64_t tail = start;
  if (kVec && start + 4 <= end) {
    const uint64_t v0 = start >> 2, vend = v0 + ((end - start) >> 2), vlast = vend - 1;
    const uint4 *s4 = (const uint4 *)a.c.src, *d4 = (const uint4 *)a.c.dst;
    const uint4 *b4 = (const uint4 *)a.c.bytes, *m4 = (const uint4 *)a.c.meta;
    const uint4 *p4 = (const uint4 *)a.c.ports, *q4 = (const uint4 *)a.c.dns;
    for (uint64_t vblk = v0; kRounds ? vblk < vend : vblk + wave0 < vend; vblk += blockDim.x) {
      const uint64_t vw = vblk + wave0;
      const bool act = vw + lane < vend;
      const uint64_t v = act ? vw + lane : vlast;
      const uint4 vs = rec_ld(&s4[v]), vd = rec_ld(&d4[v]), vm = rec_ld(&m4[v]);
      const uint4 vb = need_bytes ? b4[v] : make_uint4(0, 0, 0, 0);
      const uint4 vp = need_ports ? p4[v] : make_uint4(0, 0, 0, 0);
      const uint4 vq = need_dns ? rec_ld(&q4[v]) : make_uint4(0, 0, 0, 0);
      const uint32_t ip[8] = {vs.x, vs.y, vs.z, vs.w, vd.x, vd.y, vd.z, vd.w};
      Lk lk[8];
      if constexpr (IP::kLds) {  // 8 LDS image reads
        uint32_t sl[8];
        ipv.iv.lookup8(ip, true, sl);
#pragma unroll
        for (int k = 0; k < 8; ++k) lk[k] = sl[k] == kIplNoSlot ? none : Lk{(int32_t)sl[k], 0u};
      } else if (a.t.pre) {  // radix table: 8 prefix loads, then 8 entry loads
        uint32_t bi[8], e[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) bi[k] = radix_block(a.t, ip[k]);
#pragma unroll
        for (int k = 0; k < 8; ++k) e[k] = radix_entry(a.t, ip[k], bi[k]);
#pragma unroll
        for (int k = 0; k < 8; ++k) lk[k] = radix_pick(e[k]);
      } else {
        ulonglong2 e1[8], e2[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) e1[k] = ip_bucket(a.t, ip_h1(ip[k], a.t.seed) & a.t.mask);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          e2[k] = ip_need2(ip[k], e1[k]) ? ip_bucket(a.t, ip_h2(ip[k], a.t.seed) & a.t.mask)
                                         : make_ulonglong2(kIpEmpty, kIpEmpty);
#pragma unroll
        for (int k = 0; k < 8; ++k) lk[k] = ip_pick(ip[k], e1[k], e2[k]);
      }
      Lk ls0 = lk[0], ls1 = lk[1], ls2 = lk[2], ls3 = lk[3];
      Lk ld0 = lk[4], ld1 = lk[5], ld2 = lk[6], ld3 = lk[7];
      uint32_t s0 = vs.x, s1 = vs.y, s2 = vs.z, s3 = vs.w, d0 = vd.x, d1 = vd.y, d2 = vd.z, d3 = vd.w;
      uint32_t b0 = vb.x, b1 = vb.y, b2 = vb.z, b3 = vb.w, m0 = vm.x, m1 = vm.y, m2 = vm.z, m3 = vm.w;
      uint32_t p0 = vp.x, p1 = vp.y, p2 = vp.z, p3 = vp.w, q0 = vq.x, q1 = vq.y, q2 = vq.z, q3 = vq.w;
      if (!act) {
        ls0 = ls1 = ls2 = ls3 = ld0 = ld1 = ld2 = ld3 = none;
        m0 = m1 = m2 = m3 = kInactiveMeta;
      }
#pragma unroll 1
      for (int k = 0; k < 4; ++k) {
        f(s0, d0, b0, m0, p0, q0, ls0, ld0, act);
        s0 = s1; s1 = s2; s2 = s3; d0 = d1; d1 = d2; d2 = d3;
        b0 = b1; b1 = b2; b2 = b3; m0 = m1; m1 = m2; m2 = m3;
        p0 = p1; p1 = p2; p2 = p3; q0 = q1; q1 = q2; q2 = q3;
        ls0 = ls1; ls1 = ls2; ls2 = ls3; ld0 = ld1; ld1 = ld2; ld2 = ld3;
      }
      if (kRounds) round_end();
    }
    tail = start + ((end - start) & ~3ULL);
  }
  auto lk1 = [&](uint32_t ip) -> Lk {
    if constexpr (IP::kLds) {
      const uint32_t v = ipv.iv.lookup(ip);
      return v == kIplNoSlot ? none : Lk{(int32_t)v, 0u};
    } else {
      return ip_lookup(a.t, ip);
    }
  };
  for (uint64_t i0 = tail + wave0; i0 < end; i0 += blockDim.x) {
    const bool act = i0 + lane < end;
    const uint64_t i = act ? i0 + lane : end - 1;
    const uint32_t sip = a.c.src[i], dip = a.c.dst[i];
    f(sip, dip, need_bytes ? a.c.bytes[i] : 0u, act ? a.c.meta[i] : kInactiveMeta, need_ports ? a.c.ports[i] : 0u,
      need_dns ? a.c.dns[i] : 0u, act ? lk1(sip) : none, act ? lk1(dip) : none, act);
  }
}

// LDS setup and the once-per-workgroup flush shared by both aggregation kernels.
__device__ __forceinline__ DenseSink dense_sink_init(const KArgs &a, unsigned long long *lds) {
  for (uint32_t i = threadIdx.x; i < a.lds_bins + 64; i += blockDim.x) lds[i] = 0ULL;
  unsigned int *ctr = (unsigned int *)&lds[a.lds_bins + 64];
  for (uint32_t w = threadIdx.x; w < kMaxSpillWindows; w += blockDim.x)
    ctr[w] = a.spill && w < a.nwin ? spill_ctr0(a, w) : 0u;
  __syncthreads();
  return make_sink(a, lds, a.lds_bins, (unsigned int *)&lds[a.lds_bins + 64]);
}

__device__ __forceinline__ void dense_flush(const KArgs &a, const DenseSink &ds) {
  __syncthreads();
  // consecutive lanes -> consecutive bins: each wave-instruction adds 512 contiguous bytes
  for (uint32_t i = threadIdx.x; i < a.lds_bins; i += blockDim.x) {
    const unsigned long long v = ds.lds[i];
    if (v) {
      atomicAdd(&a.d.cnt[i], v >> kLdsCountShift);
      const unsigned long long by = v & kLdsBytesMask;
      if (by) atomicAdd(&a.d.byt[i], by);
    }
  }
  spill_counts_out(a, ds.ctr);
}

// Stores this workgroup's segment-list fills and, for device-conditional folds, adds
// its fullest list to the launch's flag (one atomic max per workgroup).
__device__ __forceinline__ void sp_counts_out(const KArgs &a, const uint32_t *sctr) {
  uint32_t mx = 0;
  for (uint32_t w = threadIdx.x; w < a.sp_nwin; w += blockDim.x) {
    const uint32_t c = sctr[w] < a.sp_cap ? sctr[w] : a.sp_cap;
    a.sp_counts[(size_t)blockIdx.x * a.sp_nwin + w] = c;
    mx = c > mx ? c : mx;
  }
  if (!a.fold_flag) return;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
  if ((threadIdx.x & 63u) == 0 && mx) atomicMax(&a.fold_flag[a.fold_parity], mx);
}

// Generic aggregation: any plan (dense, sparse, DNS, remote context, sketches).
template <bool kVec, bool kSketch>
__global__ __launch_bounds__(1024) void aggregate_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds[];
  // LDS: dense bins + extras, then the segment-list fill counters
  uint32_t *sctr = (uint32_t *)&lds[a.lds_bins + kLdsExtraWords];
  for (uint32_t i = threadIdx.x; i < a.sp_nwin; i += blockDim.x) {
    const uint32_t c0 = a.accum ? a.sp_counts[(size_t)blockIdx.x * a.sp_nwin + i] : 0u;
    sctr[i] = c0 < a.sp_cap ? c0 : a.sp_cap;
  }
  // hot-key cache after the segment counters (8-byte aligned), then the doorkeeper bitmap
  HotKey *hot = (HotKey *)&lds[a.lds_bins + kLdsExtraWords + (a.sp_nwin + 1) / 2];
  for (uint32_t i = threadIdx.x; i < a.hot_n; i += blockDim.x) hot[i].tag = 0ULL;
  uint32_t *door = (uint32_t *)(hot + a.hot_n);
  const uint32_t door_words = a.door_log2 ? 1u << (a.door_log2 - 5) : 0u;
  for (uint32_t i = threadIdx.x; i < door_words; i += blockDim.x) door[i] = 0u;
  const DenseSink ds = dense_sink_init(a, lds);  // (its barrier covers sctr, tags, bitmap)
  DevSparse s = a.s;
  // LDS pointers set unconditionally (hot_n / door_log2 = 0 disable them), so every access
  // through them compiles to ds_* instructions, not flat ones
  s.lctr = sctr;
  s.hot = hot;
  s.hot_n = a.hot_n;
  s.door = door;
  s.door_log2 = a.door_log2;
  if (a.sp_lists) {  // this workgroup's lists: compact u64 keys or wide 4- / 3-word entries
    s.lists = a.sp_lists + (size_t)blockIdx.x * a.sp_nwin * a.sp_cap * list_entry_words(s);
    s.lcap = a.sp_cap;
  }
  for_each_record<kVec>(a, a.p.need_ports || kSketch, a.p.need_dns,
                        [&](uint32_t sip, uint32_t dip, uint32_t nb, uint32_t meta, uint32_t ports,
                            uint32_t dns, const Lk &ls, const Lk &ld, bool act) {
                          apply_groups(a.p, ds, s, sip, dip, nb, meta, ports, dns, ls, ld);
                          if (kSketch && act) sketch_update(a.sk, sip, dip, ports, meta_proto(meta), ls);
                        });
  dense_flush(a, ds);  // (starts with a barrier)
  if (a.hot_n) {  // the cached keys, once per workgroup (dense_flush's barrier precedes):
    // into the segment lists with their counts, or straight into the table
    DevSparse g = s;
    g.hot_n = 0;
    for (uint32_t i = threadIdx.x; i < a.hot_n; i += blockDim.x) {
      const HotKey e = hot[i];
      if (e.tag != 2ULL) continue;
      if (g.lists) wide_append(g, key_hash(e.k0, e.k1, e.k2), e.k0, e.k1, e.k2, e.cnt, e.byt);
      else sparse_add(g, e.k0, e.k1, e.k2, e.cnt, e.byt);
    }
    __syncthreads();
  }
  sp_counts_out(a, sctr);
}

// Sparse-only plans whose 192-bit group-by keys go through the per-segment lists (remote
// context; local context with ip / port options), without tcpflags groups: the generic
// kernel's runtime plan walk, dense sink and de-duplication paths cost ~500 VALU and ~6
// SALU wave-instructions per record there (PMC, profiles/round3/t3b_pmc_c4-remote.json)
// and spilled VGPRs.  Here the group count and context are compile-time, and with kExcl
// (the groups' families are pairwise distinct, so their verdict / DNS-type tests are
// mutually exclusive) a record takes exactly one key build and one insert, whichever
// group it matches.  Insert: key hash once, doorkeeper, LDS hot-key cache, else the
// key's segment list (wide_insert).
template <int NG, bool kRemote, bool kExcl, int kIp>
__global__ __launch_bounds__(1024) void wide_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds[];
  // LDS: (kIp >= 0) the image of every pod IP, segment-list fill counters, hot-key cache
  // (8-byte aligned), doorkeeper bitmap
  const uint32_t img_words = kIp >= 0 ? a.ipl_bytes / 8 : 0u;
  if (kIp >= 0) fill_lds_u4((uint4 *)lds, (const uint4 *)a.ipl, a.ipl_bytes / 16);
  uint32_t *sctr = (uint32_t *)(lds + img_words);
  for (uint32_t i = threadIdx.x; i < a.sp_nwin; i += blockDim.x) {
    const uint32_t c0 = a.accum ? a.sp_counts[(size_t)blockIdx.x * a.sp_nwin + i] : 0u;
    sctr[i] = c0 < a.sp_cap ? c0 : a.sp_cap;
  }
  HotKey *hot = (HotKey *)&lds[img_words + (a.sp_nwin + 1) / 2];
  for (uint32_t i = threadIdx.x; i < a.hot_n; i += blockDim.x) hot[i].tag = 0ULL;
  uint32_t *door = (uint32_t *)(hot + a.hot_n);
  const uint32_t door_words = a.door_log2 ? 1u << (a.door_log2 - 5) : 0u;
  for (uint32_t i = threadIdx.x; i < door_words; i += blockDim.x) door[i] = 0u;
  __syncthreads();
  DevSparse s = a.s;
  s.lctr = sctr;
  s.hot = hot;
  s.hot_n = a.hot_n;
  s.door = door;
  s.door_log2 = a.door_log2;
  s.lists = a.sp_lists + (size_t)blockIdx.x * a.sp_nwin * a.sp_cap * list_entry_words(s);
  s.lcap = a.sp_cap;
  uint32_t fam[NG], sop[NG], dop[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    fam[g] = g < a.p.ngroups ? a.p.g[g].family : (uint32_t)FAM_COUNT;
    sop[g] = a.p.g[g].src_opts;
    dop[g] = a.p.g[g].dst_opts;
  }
  auto body = [&](uint32_t sip, uint32_t dip, uint32_t nb, uint32_t meta, uint32_t ports, uint32_t dns,
                  const Lk &ls, const Lk &ld, bool act) {
    const uint32_t proto = meta_proto(meta), verdict = meta_verdict(meta);
    const uint32_t tdir = meta_tdir(meta), reason = meta_reason(meta), dnstype = meta_dnstype(meta);
    const uint32_t sport = ports & 0xFFFFu, dport = ports >> 16;
    // the updates of group g (family f, options o1 / o2) for this record
    auto update = [&](uint32_t g, uint32_t f, uint32_t o1, uint32_t o2, bool hit) {
      const uint32_t addb = f <= FAM_DROP ? nb : 0u;
      if (kRemote) {
        const SideKey ks = side_key(o1, sip, ls, sport, proto);
        const SideKey kd = side_key(o2, dip, ld, dport, proto);
        uint32_t sub = 0, dnsv = 0;
        if (f == FAM_FWD || f == FAM_RETRANS) sub = tdir << 1;
        else if (f == FAM_DROP) sub = (reason << 3) | (tdir << 1);
        else dnsv = dns;
        if (hit)
          wide_insert(s, key0(g, sub, ks.slot1, ks.ip), key1(ks.port17, kd.port17, kd.slot1), key2(kd.ip, dnsv),
                      addb);
        return;
      }
      // getLocalCtxValues (types.go:379-416): src -> egress, dst -> ingress
      if (o1 == 0 || !hit) return;
      const bool s_ok = ls.slot >= 0 && !ls.api, d_ok = ld.slot >= 0 && !ld.api;
      if (f == FAM_DNS_REQ || f == FAM_DNS_RESP) {  // dns.go:506-540: one side
        const uint32_t side = (s_ok && d_ok) ? ((tdir == 1) ? 0u : 1u) : (d_ok ? 0u : 1u);
        const SideKey k = side == 0 ? side_key(o1, dip, ld, dport, proto) : side_key(o1, sip, ls, sport, proto);
        if (s_ok || d_ok) wide_insert(s, key0(g, side, k.slot1, k.ip), key1(k.port17, 0, 0), key2(0, dns), 0);
        return;
      }
      const uint32_t rs = f == FAM_DROP ? reason << 3 : 0u;
      if (d_ok) {
        const SideKey k = side_key(o1, dip, ld, dport, proto);
        wide_insert(s, key0(g, rs, k.slot1, k.ip), key1(k.port17, 0, 0), 0, addb);
      }
      if (s_ok) {
        const SideKey k = side_key(o1, sip, ls, sport, proto);
        wide_insert(s, key0(g, rs | 1u, k.slot1, k.ip), key1(k.port17, 0, 0), 0, addb);
      }
    };
    if (kExcl) {  // at most one group matches: its descriptors by selects
      uint32_t gs = 0, f = FAM_COUNT, o1 = 0, o2 = 0;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const bool m = family_matches(fam[g], verdict, proto, dnstype, 0u);
        gs = m ? (uint32_t)g : gs;
        f = m ? fam[g] : f;
        o1 = m ? sop[g] : o1;
        o2 = m ? dop[g] : o2;
      }
      update(gs, f, o1, o2, act && f != FAM_COUNT);
    } else {
#pragma unroll
      for (int g = 0; g < NG; ++g)
        update((uint32_t)g, fam[g], sop[g], dop[g], act && family_matches(fam[g], verdict, proto, dnstype, 0u));
    }
  };
  if constexpr (kIp >= 0) {
    const LdsIp<kIp> ipv{{(const uint8_t *)lds, a.ipl_nb, a.ipl_seed, a.ipl_npfx, a.ipl_pfx[0], a.ipl_pfx[1],
                          a.ipl_pfx[2], a.ipl_pfx[3], a.ipl_dr[0], a.ipl_dr[1], a.ipl_dr[2], a.ipl_dr[3]}};
    for_each_record<true>(a, a.p.need_ports, a.p.need_dns, body, NoRounds{}, ipv);
  } else {
    for_each_record<true>(a, a.p.need_ports, a.p.need_dns, body);
  }
  __syncthreads();
  {  // the cached keys, once per workgroup: into the segment lists with their counts
    DevSparse g = s;
    g.hot_n = 0;
    for (uint32_t i = threadIdx.x; i < a.hot_n; i += blockDim.x) {
      const HotKey e = hot[i];
      if (e.tag == 2ULL) wide_append(g, key_hash(e.k0, e.k1, e.k2), e.k0, e.k1, e.k2, e.cnt, e.byt);
    }
    __syncthreads();
  }
  sp_counts_out(a, sctr);
}

// Workgroup w folds table segment w: its 2^seg_log2 (key, count) slots are loaded into
// LDS, every aggregation workgroup's list of keys for the segment is inserted with LDS
// 64-bit CAS + add (the probe sequence of sparse_add_compact), and the segment is
// stored back -- coalesced segment traffic instead of two memory-side atomics per key.
__global__ __launch_bounds__(1024) void sparse_fold_kernel(DevSparse s, const unsigned long long *lists,
                                                           const uint32_t *counts, uint32_t n_lists,
                                                           uint32_t nwin, uint32_t cap) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long seg[];
  const uint32_t w = blockIdx.x, nslot = 1u << s.seg_log2, smask = nslot - 1u;
  ulonglong2 *g = (ulonglong2 *)(s.k0 + 2ull * ((size_t)w << s.seg_log2));
  fill_lds_u4((uint4 *)seg, (const uint4 *)g, nslot);
  __syncthreads();
  auto insert = [&](unsigned long long key) {
    const uint32_t h = compact_home(s, key);
    // the key already in its home slot (a key is published whole by its claiming CAS):
    // one read, then the no-return add.  (Reading every probe first, as the wide fold does,
    // measured slower here: a compact probe's CAS is one round trip already --
    // profiles/round6/exp/r6r_c5_*)
    if (__hip_atomic_load(&seg[2 * h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == key) {
      atomicAdd(&seg[2 * h + 1], 1ULL);
      return;
    }
    for (uint32_t probe = 0; probe <= smask; ++probe) {
      const uint32_t i = (h + probe) & smask;
      const unsigned long long cur = atomicCAS(&seg[2 * i], 0ULL, key);
      if (cur == 0ULL || cur == key) {
        atomicAdd(&seg[2 * i + 1], 1ULL);
        return;
      }
    }
    atomicAdd(s.dropped, 1ULL);
  };
  // lpl lanes per list (a power of two <= 64: the workgroup's lanes spread over the
  // lists), each taking every lpl-th key with 8 loads in flight before its inserts.  A
  // lane used to own a whole list: with one list per aggregation workgroup (256) only 4 of
  // the 16 waves worked, and after the deferred launches a list holds hundreds of keys
  // inserted one LDS round trip after another (C5: the fold grew by ~0.07 ms per launch).
  uint32_t lpl = 1;
  while (lpl < 64 && lpl * 2 * n_lists <= blockDim.x) lpl *= 2;
  const uint32_t lists_per_round = blockDim.x / lpl, sub = threadIdx.x & (lpl - 1);
  for (uint32_t l0 = 0; l0 < n_lists; l0 += lists_per_round) {
    const uint32_t l = l0 + threadIdx.x / lpl;
    if (l >= n_lists) continue;
    const uint32_t cnt = counts[(size_t)l * nwin + w];
    const unsigned long long *e = lists + ((size_t)l * nwin + w) * cap;
    uint32_t k = sub;
    for (; k + 7 * lpl < cnt; k += 8 * lpl) {
      unsigned long long v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = e[k + q * lpl];
#pragma unroll
      for (int q = 0; q < 8; ++q) insert(v[q]);
    }
    for (; k < cnt; k += lpl) insert(e[k]);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nslot; i += blockDim.x) g[i] = ((const ulonglong2 *)seg)[i];
}

// Workgroup w folds wide-key table segment w (2^seg_log2 slots of k0 k1 k2 cnt byt): the
// segment is loaded into LDS (field-major, so probes of consecutive slots hit consecutive
// banks), every aggregation workgroup's list of entries for the segment is inserted with
// LDS 64-bit CAS / adds -- the probe sequence and claim / publish protocol of sparse_add
// (a lane that meets a key still being published moves on, so a key may take two slots;
// the host sums them) -- and the segment is stored back.  Segments no list reaches are
// not touched.
// re-reads of a slot whose key (same k0) is being published before probing on: a claimer
// publishes within a few instructions, and the bound keeps every insert finite even if
// the compiler defers the claimer's stores past the loop
constexpr uint32_t kFoldSpin = 32;
constexpr uint32_t kFoldSegLoads = 10;  // 16-byte segment loads per lane in flight (5 * 2^12 / 2 / 1024)
__global__ __launch_bounds__(1024) void sparse_fold_wide_kernel(DevSparse s, const unsigned long long *lists,
                                                                uint32_t *counts, uint32_t n_lists,
                                                                uint32_t nwin, uint32_t cap, uint32_t *flag,
                                                                uint32_t parity, uint32_t thr) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long seg[];
  const uint32_t w = blockIdx.x, N = 1u << s.seg_log2, smask = N - 1u;
  if (flag) {
    // device-conditional fold: the next launch's flag starts at 0; while the fullest list
    // of the launches since the last fold is below thr, the lists keep growing (the next
    // aggregation launch appends after them).  Atomics: executed at memory, so no XCD's
    // L2 can hold a stale copy of the flags.
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicExch(&flag[parity ^ 1u], 0u);
    if (thr && atomicOr(&flag[parity], 0u) < thr) return;  // the same value for every workgroup
  }
  // lanes per list: the workgroup's threads spread over the lists (a power of two <= 64)
  uint32_t lpl = 1;
  while (lpl < 64 && lpl * 2 * n_lists <= blockDim.x) lpl *= 2;
  const uint32_t lists_per_round = blockDim.x / lpl, sub = threadIdx.x & (lpl - 1);
  // Per-segment decision: a device-conditional fold (thr > 0) folds only the segments with
  // a list at thr or beyond; the others keep their lists (and fill counters) for a later
  // fold, so a segment's 160 KiB pass in and out is paid when its lists are long -- not in
  // every launch for every segment because one workgroup's list of one segment filled
  // (C4-remote: a few hot flows miss their cache ways in some workgroups every launch).
  // (a flag word in the segment's LDS: __syncthreads_or would take static LDS beyond the
  // 160 KiB the segment may fill)
  uint32_t mx = 0;
  for (uint32_t l = threadIdx.x; l < n_lists; l += blockDim.x) mx = max(mx, counts[(size_t)l * nwin + w]);
  if (threadIdx.x == 0) seg[0] = 0ULL;
  __syncthreads();
  if (thr ? mx >= thr : mx != 0u) seg[0] = 1ULL;
  __syncthreads();
  const bool work = seg[0] != 0ULL;
  __syncthreads();
  if (!work) return;
  unsigned long long *K0 = seg, *K1 = seg + N, *K2 = seg + 2 * N, *CN = seg + 3 * N, *BY = seg + 4 * N;
  unsigned long long *g = s.k0 + (size_t)kSparseSlotWords * ((size_t)w << s.seg_log2);
  // the segment in 16-byte words (N is even: 5 * N / 2 of them, 16-byte aligned), up to 10
  // loads per lane in flight -- the whole 160 KiB segment in one round trip at 1024 lanes
  // -- then scattered field-major into LDS
  const uint32_t nv = kSparseSlotWords * N / 2;
  auto field = [&](uint32_t word) -> unsigned long long & {
    const uint32_t slot = word / kSparseSlotWords;
    return seg[(word - slot * kSparseSlotWords) * N + slot];
  };
  for (uint32_t v0 = threadIdx.x; v0 < nv; v0 += kFoldSegLoads * blockDim.x) {
    ulonglong2 v[kFoldSegLoads];
#pragma unroll
    for (uint32_t q = 0; q < kFoldSegLoads; ++q) {
      const uint32_t j = v0 + q * blockDim.x;
      if (j < nv) v[q] = ((const ulonglong2 *)g)[j];
    }
#pragma unroll
    for (uint32_t q = 0; q < kFoldSegLoads; ++q) {
      const uint32_t j = v0 + q * blockDim.x;
      if (j < nv) {
        field(2 * j) = v[q].x;
        field(2 * j + 1) = v[q].y;
      }
    }
  }
  __syncthreads();
  auto insert = [&](uint32_t h, uint64_t x0, uint64_t x1, uint64_t x2, uint64_t c, uint64_t b) {  // h: home slot
    // Every probe first reads the slot: K2, then K0 and K1, issued together (atomic loads
    // keep their program order; LDS executes a wave's accesses in order and a claimer
    // publishes K2 after K1, so a published K2 means the K0 / K1 read after it are final).  A key already in
    // the segment -- every key once the same flows come back -- costs one LDS round trip
    // per probe and no-return adds; only a free slot takes the CAS claim.  (The claim CAS
    // on every probe, then two dependent reads, made each probe three round trips, and a
    // wave waits for its longest probe run: profiles/round6/exp/r6q_*.)
    uint32_t spin = 0;
    for (uint32_t probe = 0; probe < N;) {
      const uint32_t i = (h + probe) & smask;
      const unsigned long long p2 = __hip_atomic_load(&K2[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const unsigned long long p0 = __hip_atomic_load(&K0[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const unsigned long long p1 = __hip_atomic_load(&K1[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (p2 == x2 && p0 == x0 && p1 == x1) {
        __hip_atomic_fetch_add(&CN[i], (unsigned long long)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (b) __hip_atomic_fetch_add(&BY[i], (unsigned long long)b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return;
      }
      if (p0 == 0ULL) {
        const unsigned long long cur = atomicCAS(&K0[i], 0ULL, (unsigned long long)x0);
        if (cur == 0ULL) {
          K1[i] = x1;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __hip_atomic_store(&K2[i], (unsigned long long)x2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // publish
          atomicAdd(&CN[i], (unsigned long long)c);
          if (b) atomicAdd(&BY[i], (unsigned long long)b);
          return;
        }
        // claimed this instant by a lane with the same k0: read the slot again
        if (cur == x0 && spin < kFoldSpin) {
          ++spin;
          continue;
        }
      } else if (p0 == x0 && p2 == kKeyPending && spin < kFoldSpin) {
        // a key with this k0 still being published: wait for it (bounded) rather than
        // claiming a second slot -- many lanes meeting one new key used to take a slot each
        ++spin;
        continue;
      }
      ++probe;
    }
    atomicAdd(s.dropped, (unsigned long long)c);
  };
  // (more than 256 lists: lpl lanes per list, each taking every lpl-th entry; a lane loads 4
  // entries before inserting any, so the list reads are in flight together instead of one
  // HBM round trip per entry)
  auto ins = [&](const ulonglong2 &a0, const ulonglong2 &a1) {
    insert((uint32_t)(a1.y >> kWideHomeShift) & smask, a0.x, a0.y, a1.x,
           (a1.y >> kWideCountShift) & ((1ULL << (kWideHomeShift - kWideCountShift)) - 1),
           a1.y & ((1ULL << kWideCountShift) - 1));
  };
  const uint32_t ew = s.narrow ? kWideNarrowWords : kWideEntryWords;
  if (n_lists <= 256) {
    // Balanced: the segment's lists as one concatenated run of E entries, dealt out in
    // 64-entry chunks round-robin over the waves (lane = offset in the chunk), so every
    // lane inserts ~E / 1024 entries however uneven the lists are -- deferred lists are,
    // and lanes fixed to a list waited on the longest -- and consecutive lanes read
    // consecutive entries.  Each wave holds the lists' prefix sums in registers (4 lists a
    // lane): inc[q] ends list 4 * lane + q inside the lane's run, which starts at B.  (Many
    // lanes then meet one new hot key at once; the probe's bounded wait on a key being
    // published keeps that key in one slot.)
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
    // entry j0 + lane of the run (wave-converged): its list's words
    auto locate = [&](uint32_t j0, bool valid) -> const unsigned long long * {
      const uint32_t j = j0 + lane;
      uint32_t L = (uint32_t)__popcll(__ballot(B <= j0)) - 1u;  // B is nondecreasing
      for (;;) {  // a chunk spans few lanes' runs
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
    for (uint32_t c0 = wv; c0 < nchunk; c0 += 4 * nwv) {  // 4 chunks' loads in flight
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
  for (uint32_t l0 = 0; l0 < n_lists; l0 += lists_per_round) {
    const uint32_t l = l0 + threadIdx.x / lpl;
    if (l >= n_lists) continue;
    const uint32_t cnt = counts[(size_t)l * nwin + w];
    if (s.narrow) {  // 3-word entries (k0, d_slot1 << 32 | d_ip, meta): three 8-byte loads
      const unsigned long long *e = lists + ((size_t)l * nwin + w) * cap * kWideNarrowWords;
      auto insn = [&](uint64_t x0, uint64_t n, uint64_t m) {
        ins(make_ulonglong2(x0, wide_unpack1(n)), make_ulonglong2(wide_unpack2(n), m));
      };
      uint32_t k = sub;
      for (; k + 3 * lpl < cnt; k += 4 * lpl) {
        unsigned long long v[12];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int j = 0; j < 3; ++j) v[3 * q + j] = e[3 * (size_t)(k + q * lpl) + j];
#pragma unroll
        for (int q = 0; q < 4; ++q) insn(v[3 * q], v[3 * q + 1], v[3 * q + 2]);
      }
      for (; k < cnt; k += lpl) insn(e[3 * (size_t)k], e[3 * (size_t)k + 1], e[3 * (size_t)k + 2]);
      continue;
    }
    const ulonglong2 *e = (const ulonglong2 *)(lists + ((size_t)l * nwin + w) * cap * kWideEntryWords);
    uint32_t k = sub;
    for (; k + 3 * lpl < cnt; k += 4 * lpl) {
      ulonglong2 v[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[2 * q] = e[2 * (k + q * lpl)];
        v[2 * q + 1] = e[2 * (k + q * lpl) + 1];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) ins(v[2 * q], v[2 * q + 1]);
    }
    for (; k < cnt; k += lpl) ins(e[2 * k], e[2 * k + 1]);
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < nv; j += blockDim.x)
    ((ulonglong2 *)g)[j] = make_ulonglong2(field(2 * j), field(2 * j + 1));
  // this segment's lists are folded: empty them for the launches that append next
  for (uint32_t l = threadIdx.x; l < n_lists; l += blockDim.x) counts[(size_t)l * nwin + w] = 0u;
}

// Dense local-context fast path: every group is endpoint-keyed (forward / drop /
// tcpflags / tcpretrans with namespace|podname|workload|service options) or, with kDns,
// a DNS group of the compact plan (its key fits 64 bits: group|side|slot|dns id, appended
// to the table segment's list as the generic kernel does).  The NG group descriptors are
// compile-time indexed, so they live in SGPRs for the whole kernel; bin arithmetic is
// 32-bit.  kDns keeps C5 (tcpflags + retransmissions + DNS at 100k pods) off the generic
// kernel's per-group dispatch.
template <int NG, bool kVec, bool kDns, uint32_t SIG = 0, bool kStage = false>
__global__ __launch_bounds__(1024) void dense_local_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds[];
  uint32_t *sctr = (uint32_t *)&lds[a.lds_bins + kLdsExtraWords];
  CompactLists cl{};
  if (kDns) {  // segment-list fill counters after the dense bins (aggregate_kernel's layout)
    for (uint32_t i = threadIdx.x; i < a.sp_nwin; i += blockDim.x) {
      const uint32_t c0 = a.accum ? a.sp_counts[(size_t)blockIdx.x * a.sp_nwin + i] : 0u;
      sctr[i] = c0 < a.sp_cap ? c0 : a.sp_cap;
    }
    cl = CompactLists{a.sp_lists + (size_t)blockIdx.x * a.sp_nwin * a.sp_cap, sctr, a.sp_cap, a.s.k0,
                      a.s.dropped, a.s.mask, a.s.seg_log2};
  }
  // kStage: spill appends are staged in per-window LDS rings (after the segment
  // counters: [nwin] round counters, then [nwin][kSpillRing] entries) and written out
  // every few steps as contiguous runs -- C5's ~1.4 appends per record to 220 windows were
  // scattered 4-byte stores (PMC: 3.2x the list bytes written).  rc[w] counts window w's
  // appends since the last flush, so an append's ring slot is what its LDS atomic returns
  // (one LDS round trip); ds.ctr[w] holds the list length at the last flush.
  uint32_t *rc = sctr + (kDns ? a.sp_nwin : 0u);
  uint32_t *ring = rc + a.nwin;
  if (kStage)
    for (uint32_t w = threadIdx.x; w < a.nwin; w += blockDim.x) rc[w] = 0u;
  const DenseSink ds = dense_sink_init(a, lds);  // (its barrier covers sctr and rc too)
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const uint32_t dummy = a.lds_bins + lane;  // absorbs predicated-off updates, never flushed
  const uint32_t wmask = (1u << a.win_shift) - 1u;
  // an entry of window w that cannot be listed: its updates as global atomics (exact)
  auto entry_global = [&](uint32_t w, uint32_t e) {
    const uint32_t bin = a.spill_lo + (w << a.win_shift) + (e & wmask);
    if (e >> 31) {
      for (uint32_t m = (e >> a.win_shift) & 0xFFu; m; m &= m - 1)
        atomicAdd(&a.d.cnt[bin + __builtin_ctz(m)], 1ULL);
      return;
    }
    atomicAdd(&a.d.cnt[bin], 1ULL);
    if (e >> a.win_shift) atomicAdd(&a.d.byt[bin], (unsigned long long)(e >> a.win_shift));
  };
  auto spill_e = [&](uint32_t w, uint32_t e) {  // kStage
    const uint32_t p = atomicAdd(&rc[w], 1u);
    if (p < kSpillRing) {
      ring[w * kSpillRing + p] = e;
      return;
    }
    const uint32_t lp = ds.ctr[w] + p;  // past the ring: straight into the list
    if (lp < ds.spill_cap) ds.spill[mul_u24(w, ds.spill_cap) + lp] = e;
    else entry_global(w, e);
  };
  auto spill = [&](uint32_t bin, uint32_t nbytes) {
    if (!kStage) {
      ds.spill_add(bin, nbytes);
      return;
    }
    spill_e(ds.window(bin), ds.entry(bin, nbytes));
  };
  // a spilled tcpflags row (8 bins, 8-aligned in its window): one entry for the whole flag
  // mask (kSpillRowMask) instead of one per flag
  const bool rows = kStage && a.row_masks;
  auto spill_row = [&](uint32_t row, uint32_t m) {
    spill_e(ds.window(row), ((row - a.spill_lo) & wmask) | (m << a.win_shift) | kSpillRowMask);
  };
  // each window's staged run to its list at the length of the last flush (all threads,
  // between barriers); a wave takes 4 windows at a time and issues all their LDS reads
  // (counters, then the <= kSpillRing = 2 x 64 staged entries per window) before its
  // global stores
  static_assert(kSpillRing == 128, "two ring entries per lane and window");
  auto flush = [&]() {
    const uint32_t wv = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    for (uint32_t w0 = wv; w0 < a.nwin; w0 += 4 * nwaves) {
      uint32_t n[4], b[4], v[4][2];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t w = w0 + q * nwaves;
        n[q] = w < a.nwin ? rc[w] : 0u;
        b[q] = w < a.nwin ? ds.ctr[w] : 0u;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const uint32_t p = lane + 64u * it;
          v[q][it] = p < min(n[q], kSpillRing) ? ring[(w0 + q * nwaves) * kSpillRing + p] : 0u;
        }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t w = w0 + q * nwaves;
        if (w >= a.nwin) continue;
        uint32_t *dst = ds.spill + mul_u24(w, ds.spill_cap);
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const uint32_t p = lane + 64u * it;
          if (p >= min(n[q], kSpillRing)) continue;
          if (b[q] + p < ds.spill_cap) dst[b[q] + p] = v[q][it];
          else entry_global(w, v[q][it]);
        }
        if (lane == 0) {
          ds.ctr[w] = b[q] + n[q];
          rc[w] = 0u;
        }
      }
    }
  };
  // flush every kStageSteps steps: ~100 appends per window on average into the 128-entry
  // rings (the excess of a busy window is stored directly); every 1 / 2 / 3 / 4 / 6 steps
  // measured 0.231 / 0.207 / 0.201 / 0.196 / 0.199 ms at C5 (profiles/round2/r5f_*, r6f_*)
  constexpr uint32_t kStageSteps = 4;
  uint32_t steps = 0;  // block-uniform
  auto round_end = [&]() {
    if (++steps % kStageSteps) return;
    __syncthreads();
    flush();
    __syncthreads();
  };

  const int ng = a.p.ngroups;
  uint32_t fam[NG], base[NG], nsub[NG], keyed[NG], sopts[NG];
  bool inl[NG];
  bool any_flags = false;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if (SIG) {  // family and LDS residency fixed at compile time (see tier1_signature)
      const uint32_t code = (SIG >> (4 * g)) & 7u;
      fam[g] = code ? code - 1 : (uint32_t)FAM_COUNT;
      inl[g] = (SIG >> (4 * g + 3)) & 1u;
    } else {
      fam[g] = g < ng ? a.p.g[g].family : (uint32_t)FAM_COUNT;
      inl[g] = a.p.g[g].dense_base + a.p.g[g].nbins <= a.lds_bins;  // whole group in the LDS window
    }
    base[g] = (uint32_t)a.p.g[g].dense_base;
    nsub[g] = a.p.g[g].nsub;
    keyed[g] = a.p.g[g].key_mode;
    sopts[g] = a.p.g[g].src_opts;
    any_flags |= fam[g] == FAM_TCPFLAGS;
  }
  for_each_record<kVec, kStage>(a, false, kDns,
                        [&](uint32_t sip, uint32_t dip, uint32_t nb, uint32_t meta, uint32_t, uint32_t dns,
                            const Lk &ls, const Lk &ld, bool) {
    const uint32_t proto = meta_proto(meta), verdict = meta_verdict(meta), reason = meta_reason(meta);
    const bool s_ok = ls.slot >= 0 && !ls.api;  // getLocalCtxValues (types.go:379-416)
    const bool d_ok = ld.slot >= 0 && !ld.api;
    const bool big = nb >= kLdsByteLimit;       // bytes of such packets go to global atomics
    const uint32_t flagmask = (any_flags && verdict == kVerdictForwarded && proto == 6)
                                  ? flag_label_mask(meta_flags(meta)) : 0u;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const uint32_t f = fam[g];
      if (f == FAM_COUNT) continue;
      if (kDns && (f == FAM_DNS_REQ || f == FAM_DNS_RESP)) {
        // dns.go:506-540: exactly one update; both sides -> pick by TrafficDirection.
        // Compact plan: no ip / port option, so the side tuple is the endpoint only.
        if (sopts[g] == 0) continue;
        const bool hit = verdict == kVerdictDns && meta_dnstype(meta) == (f == FAM_DNS_REQ ? kDnsQuery : kDnsResponse);
        const uint32_t side = (s_ok && d_ok) ? (meta_tdir(meta) == 1 ? 0u : 1u) : (d_ok ? 0u : 1u);
        const SideKey k = side == 0 ? side_key(sopts[g], dip, ld, 0u, proto) : side_key(sopts[g], sip, ls, 0u, proto);
        if (hit && (s_ok || d_ok)) cl.insert(key0((uint32_t)g, side, k.slot1, k.ip) | (uint64_t)dns);
        continue;
      }
      const uint32_t kd = keyed[g] ? (uint32_t)ld.slot : 0u, ks = keyed[g] ? (uint32_t)ls.slot : 0u;
      // slots < 2^16, nsub <= 64: 24-bit multiplies (full rate)
      const uint32_t row_d = base[g] + mul_u24(kd * 2u, nsub[g]);        // side 0: ingress (dst)
      const uint32_t row_s = base[g] + mul_u24(ks * 2u + 1u, nsub[g]);   // side 1: egress (src)
      if (f == FAM_TCPFLAGS) {
        uint32_t m = flagmask;
        if (inl[g]) {
          while (__ballot(m != 0)) {  // trips = most flags any lane of the wave has
            const bool v = m != 0;
            const uint32_t bit = v ? (uint32_t)__builtin_ctz(m) : 0u;
            atomicAdd(&lds[v && d_ok ? row_d + bit : dummy], kLdsCountOne);
            atomicAdd(&lds[v && s_ok ? row_s + bit : dummy], kLdsCountOne);
            m &= m - 1;
          }
        } else if (rows) {
          if (m && d_ok) spill_row(row_d, m);
          if (m && s_ok) spill_row(row_s, m);
        } else {
          for (; m; m &= m - 1) {
            const uint32_t bit = (uint32_t)__builtin_ctz(m);
            if (d_ok) spill(row_d + bit, 0);
            if (s_ok) spill(row_s + bit, 0);
          }
        }
        continue;
      }
      bool hit;
      if (f == FAM_FWD) hit = verdict == kVerdictForwarded;
      else if (f == FAM_DROP) hit = verdict == kVerdictDropped;
      else hit = verdict == kVerdictRetrans;
      const uint32_t sub = f == FAM_DROP ? reason : 0u;
      const uint32_t add_b = f <= FAM_DROP ? nb : 0u;
      if (inl[g]) {
        const unsigned long long val = kLdsCountOne | (big ? 0u : add_b);
        atomicAdd(&lds[hit && d_ok ? row_d + sub : dummy], val);
        atomicAdd(&lds[hit && s_ok ? row_s + sub : dummy], val);
        if (big && hit && add_b) {
          if (d_ok) atomicAdd(&a.d.byt[row_d + sub], (unsigned long long)add_b);
          if (s_ok) atomicAdd(&a.d.byt[row_s + sub], (unsigned long long)add_b);
        }
      } else if (hit) {
        if (d_ok) spill(row_d + sub, add_b);
        if (s_ok) spill(row_s + sub, add_b);
      }
    }
  }, round_end);
  if (kStage) {  // the tail records' staged entries
    __syncthreads();
    flush();
  }
  dense_flush(a, ds);  // (starts with a barrier)
  if (kDns)
    for (uint32_t w = threadIdx.x; w < a.sp_nwin; w += blockDim.x)
      a.sp_counts[(size_t)blockIdx.x * a.sp_nwin + w] = sctr[w] < a.sp_cap ? sctr[w] : a.sp_cap;
}

// ---- tier-1: IP table and 32-bit bins both in LDS -------------------------------------
struct L4Ctx {
  uint32_t *bins;  // [L4] u32 bins, then 64 dummies, then the spill-window counters
  uint32_t dummy;  // this lane's dummy word: absorbs predicated-off updates
  DevDense d;
  // Does the add of (count 1, bytes nb) that returned `old` need fix()?  Branch-free:
  // callers OR this over all their adds and take the slow path once per wave.
  static __device__ __forceinline__ bool fix_needed(bool valid, uint32_t old, uint32_t nb) {
    const uint32_t b = nb < kL4ByteLimit ? nb : 0u;
    return valid & (((old & kL4BytesMask) + b > kL4BytesMask) | (old >= 0xFFE00000u) |
                    (nb >= kL4ByteLimit));
  }
  // Exact correction after a packed add (count:12 | bytes:20) returned `old`: a carry
  // out of the bytes field, a wrap of the count field, or a packet too big for the
  // field is booked into the global counters.  Rare; the test is 3 VALU ops.
  __device__ __forceinline__ void fix(bool valid, uint32_t old, uint32_t nb, uint32_t bin) const {
    const uint32_t b = nb < kL4ByteLimit ? nb : 0u;
    if (!(valid && ((old & kL4BytesMask) + b > kL4BytesMask || old >= 0xFFE00000u ||
                    nb >= kL4ByteLimit)))
      return;
    if (nb >= kL4ByteLimit) atomicAdd(&d.byt[bin], (unsigned long long)nb);
    const uint32_t carry = ((old & kL4BytesMask) + b) >> kL4CountShift;
    const uint32_t wrap = ((old >> kL4CountShift) + 1u + carry) >> (32 - kL4CountShift);
    if (carry) {
      atomicAdd(&d.byt[bin], (unsigned long long)kL4ByteLimit);
      atomicAdd(&d.cnt[bin], ~0ULL);  // the carry also bumped the count field
    }
    if (wrap) atomicAdd(&d.cnt[bin], 1ULL << (32 - kL4CountShift));
  }
};
static_assert(kL4CountShift == 20, "fix() thresholds assume count:12 | bytes:20");

// Group descriptors of the dense local-context plan, compile-time indexed (SGPRs).
// SIG != 0 also fixes every group's family and LDS residency at compile time (4 bits per
// group: family + 1, bit 3 = in LDS; see tier1_signature), so the per-record family
// dispatch folds away; SIG == 0 reads them from the plan.
template <int NG, uint32_t SIG>
struct DenseGroups {
  uint32_t fam[NG], base[NG], nsub[NG], keyed[NG];
  bool inl[NG];
  bool any_flags;
  bool any_spilled;  // some group's bins are outside LDS
  __device__ __forceinline__ DenseGroups(const Plan &p, uint32_t L) {
    any_flags = false;
    any_spilled = false;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (SIG) {
        const uint32_t code = (SIG >> (4 * g)) & 7u;
        fam[g] = code ? code - 1 : (uint32_t)FAM_COUNT;
        inl[g] = (SIG >> (4 * g + 3)) & 1u;
      } else {
        fam[g] = g < p.ngroups ? p.g[g].family : (uint32_t)FAM_COUNT;
        inl[g] = p.g[g].dense_base + p.g[g].nbins <= L;
      }
      base[g] = (uint32_t)p.g[g].dense_base;
      nsub[g] = p.g[g].nsub;
      keyed[g] = p.g[g].key_mode;
      any_flags |= fam[g] == FAM_TCPFLAGS;
      any_spilled |= fam[g] != FAM_COUNT && !inl[g];
    }
  }
};

// Does a record update group f (tier-1 families only: fwd / drop / tcpflags / retrans)?
__device__ __forceinline__ bool fam_hit(uint32_t f, uint32_t verdict, uint32_t flagmask) {
  if (f == FAM_TCPFLAGS) return flagmask != 0;
  return verdict == (f == FAM_FWD ? kVerdictForwarded : f == FAM_DROP ? kVerdictDropped : kVerdictRetrans);
}

// Wave-level compaction queue for the records that update a spilled group (one whose
// bins are not in LDS).  Such records are rare (C2: the 10 % drops), so updating them
// in place would issue every spill instruction for ~5 active lanes of 64.  Instead each
// step pushes them into three queue registers (one entry per lane) with ds_permute --
// LDS crossbar, no LDS memory -- and the spill code runs once per 64 queued records
// with every lane busy.  Push = ballot + mbcnt + a bijective lane permutation: hits go
// to queue positions [n, n + hits), misses to the remaining ones, so every lane
// receives exactly one value.
struct SpillQ {
  uint32_t e0, e1, e2;  // queued entries: slots (ss | sd << 16), bytes, meta
  uint32_t n;           // queued entries (wave-uniform), lanes [0, n)
  uint32_t r0, r1, r2;  // this push's permuted values (wrap-around part on overflow)
  // push; returns true when the queue holds 64 entries (caller flushes, then next())
  __device__ __forceinline__ bool push(bool v, uint32_t lane, uint32_t a0, uint32_t a1, uint32_t a2) {
    const uint64_t m = __ballot(v);
    const uint32_t cnt = (uint32_t)__popcll(m);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const uint32_t pos = v ? n + below : n + cnt + (lane - below);
    const int addr = (int)((pos & 63u) << 2);
    r0 = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)a0);
    r1 = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)a1);
    r2 = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)a2);
    const bool got = lane >= n && lane < n + cnt;
    e0 = got ? r0 : e0;
    e1 = got ? r1 : e1;
    e2 = got ? r2 : e2;
    n += cnt;
    return n >= 64;
  }
  // push of two values (the third register is left alone)
  __device__ __forceinline__ bool push2(bool v, uint32_t lane, uint32_t a0, uint32_t a1) {
    const uint64_t m = __ballot(v);
    const uint32_t cnt = (uint32_t)__popcll(m);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const uint32_t pos = v ? n + below : n + cnt + (lane - below);
    const int addr = (int)((pos & 63u) << 2);
    r0 = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)a0);
    r1 = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)a1);
    const bool got = lane >= n && lane < n + cnt;
    e0 = got ? r0 : e0;
    e1 = got ? r1 : e1;
    n += cnt;
    return n >= 64;
  }
  // after flushing a full queue: the wrapped entries become the queue
  __device__ __forceinline__ void next() { e0 = r0; e1 = r1; e2 = r2; n -= 64; }
};

// R records of one thread through every group (tier-1).  Group-outer / record-inner:
// a group's 2R returning LDS adds are all issued before any result is inspected, so
// their latency overlaps.  ss/sd: source / destination slot or kIplNoSlot.
// kMode: 0 every group; 1 LDS groups only (spilled ones go through SpillQ); 2 spilled
// groups only (the SpillQ flush).
template <int NG, uint32_t SIG, int R, int kMode = 0>
__device__ __forceinline__ void l4_records(const DenseGroups<NG, SIG> &G, const L4Ctx &l4,
                                           const DenseSink &ds, const uint32_t (&nbytes)[R],
                                           const uint32_t (&meta)[R], const uint32_t (&ss)[R],
                                           const uint32_t (&sd)[R]) {
  uint32_t verdict[R], reason[R], flagmask[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    verdict[k] = meta_verdict(meta[k]);
    reason[k] = meta_reason(meta[k]);
    flagmask[k] = (G.any_flags && verdict[k] == kVerdictForwarded && meta_proto(meta[k]) == 6)
                      ? flag_label_mask(meta_flags(meta[k])) : 0u;
  }
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const uint32_t f = G.fam[g];
    if (f == FAM_COUNT) continue;
    if ((kMode == 1 && !G.inl[g]) || (kMode == 2 && G.inl[g])) continue;
    uint32_t rd[R], rs[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {  // slots < 2^16, nsub <= 64: 24-bit multiplies
      const uint32_t kd = G.keyed[g] ? sd[k] : 0u, ks = G.keyed[g] ? ss[k] : 0u;
      rd[k] = G.base[g] + mul_u24(kd * 2u, G.nsub[g]);       // side 0: ingress (dst)
      rs[k] = G.base[g] + mul_u24(ks * 2u + 1u, G.nsub[g]);  // side 1: egress (src)
    }
    if (f == FAM_TCPFLAGS) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        uint32_t m = flagmask[k];
        const bool d_ok = sd[k] != kIplNoSlot, s_ok = ss[k] != kIplNoSlot;
        if (G.inl[g]) {
          while (__ballot(m != 0)) {
            const bool v = m != 0;
            const uint32_t bit = v ? (uint32_t)__builtin_ctz(m) : 0u;
            atomicAdd(&l4.bins[v && d_ok ? rd[k] + bit : l4.dummy], 1u);
            atomicAdd(&l4.bins[v && s_ok ? rs[k] + bit : l4.dummy], 1u);
            m &= m - 1;
          }
        } else {
          for (; m; m &= m - 1) {
            const uint32_t bit = (uint32_t)__builtin_ctz(m);
            if (d_ok) ds.spill_add(rd[k] + bit, 0);
            if (s_ok) ds.spill_add(rs[k] + bit, 0);
          }
        }
      }
      continue;
    }
    const uint32_t want = f == FAM_FWD ? kVerdictForwarded : f == FAM_DROP ? kVerdictDropped
                                                                          : kVerdictRetrans;
    bool vd[R], vs[R];
    uint32_t bd[R], bs[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const bool hit = verdict[k] == want;
      const uint32_t sub = f == FAM_DROP ? reason[k] : 0u;
      vd[k] = hit & (sd[k] != kIplNoSlot);  // '&': no short-circuit branches
      vs[k] = hit & (ss[k] != kIplNoSlot);
      bd[k] = rd[k] + sub;
      bs[k] = rs[k] + sub;
    }
    if (G.inl[g]) {
      if (f <= FAM_DROP) {
        uint32_t od[R], os[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const uint32_t add = (1u << kL4CountShift) | (nbytes[k] < kL4ByteLimit ? nbytes[k] : 0u);
          od[k] = atomicAdd(&l4.bins[vd[k] ? bd[k] : l4.dummy], add);
          os[k] = atomicAdd(&l4.bins[vs[k] ? bs[k] : l4.dummy], add);
        }
        bool need = false;
#pragma unroll
        for (int k = 0; k < R; ++k)
          need |= L4Ctx::fix_needed(vd[k], od[k], nbytes[k]) | L4Ctx::fix_needed(vs[k], os[k], nbytes[k]);
        if (__builtin_expect(__ballot(need) != 0, 0)) {  // rare: a carry, a wrap or a jumbo size
#pragma unroll
          for (int k = 0; k < R; ++k) {
            l4.fix(vd[k], od[k], nbytes[k], bd[k]);
            l4.fix(vs[k], os[k], nbytes[k], bs[k]);
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < R; ++k) {
          atomicAdd(&l4.bins[vd[k] ? bd[k] : l4.dummy], 1u);
          atomicAdd(&l4.bins[vs[k] ? bs[k] : l4.dummy], 1u);
        }
      }
    } else if (ds.spill) {
      // spilled group: reserve all 2R list positions first (dummy word for lanes
      // without an update), then store
      uint32_t wd[R], ws[R], pd[R], ps[R];
#pragma unroll
      for (int k = 0; k < R; ++k) {
        wd[k] = ds.window(bd[k]);
        ws[k] = ds.window(bs[k]);
        if (kMode == 2) {  // SpillQ flush: converged wave
          pd[k] = wave_reserve(vd[k], wd[k], ds.ctr, ds.wbits);
          ps[k] = wave_reserve(vs[k], ws[k], ds.ctr, ds.wbits);
        } else {
          pd[k] = atomicAdd(vd[k] ? &ds.ctr[wd[k]] : &l4.bins[l4.dummy], 1u);
          ps[k] = atomicAdd(vs[k] ? &ds.ctr[ws[k]] : &l4.bins[l4.dummy], 1u);
        }
      }
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const uint32_t add_b = f <= FAM_DROP ? nbytes[k] : 0u;
        if (vd[k]) ds.spill_put(bd[k], wd[k], pd[k], add_b);
        if (vs[k]) ds.spill_put(bs[k], ws[k], ps[k], add_b);
      }
    } else {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const uint32_t add_b = f <= FAM_DROP ? nbytes[k] : 0u;
        if (vd[k]) ds.spill_add(bd[k], add_b);
        if (vs[k]) ds.spill_add(bs[k], add_b);
      }
    }
  }
}

template <int NG, bool kVec, uint32_t SIG, int kIp>
__global__ __launch_bounds__(1024) void dense_lds_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const IplView<kIp> iv{smem,          a.ipl_nb,     a.ipl_seed,   a.ipl_npfx,   a.ipl_pfx[0], a.ipl_pfx[1],
                        a.ipl_pfx[2],  a.ipl_pfx[3], a.ipl_dr[0],  a.ipl_dr[1],  a.ipl_dr[2],  a.ipl_dr[3]};
  uint32_t *bins = (uint32_t *)(smem + a.ipl_bytes);
  const uint32_t L4 = a.lds_bins;
  fill_lds_u4((uint4 *)smem, (const uint4 *)a.ipl, a.ipl_bytes / 16);
  if (a.stage_accum) {  // deferred reduce: continue from this workgroup's staged copy
    const uint32_t *mine = a.stage_a + (size_t)blockIdx.x * a.stage_a_stride;
    for (uint32_t i = threadIdx.x; i < L4 + 64; i += blockDim.x) bins[i] = i < L4 ? mine[i] : 0u;
  } else {
    for (uint32_t i = threadIdx.x; i < L4 + 64; i += blockDim.x) bins[i] = 0u;
  }
  for (uint32_t w = threadIdx.x; w < kMaxSpillWindows; w += blockDim.x)
    bins[L4 + 64 + w] = a.spill && w < a.nwin ? spill_ctr0(a, w) : 0u;
  __syncthreads();
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const L4Ctx l4{bins, L4 + lane, a.d};
  const DenseSink ds = make_sink(a, nullptr, 0, bins + L4 + 64);
  const DenseGroups<NG, SIG> G(a.p, L4);
  SpillQ q{};
  // C2's signature spills only the drop group (group 1): a queued record is its slots and
  // bytes | reason << 29 -- two registers (one ds_permute fewer per record); the meta word
  // is rebuilt at the flush.  Bytes >= 2^29 are added to the drop bins at the push.
  constexpr bool kDropQ = SIG == kSigFwdLdsDropSpill;
  constexpr uint32_t kQBytes = (1u << 29) - 1u;
  // spill updates of the queued records; lanes >= n (final partial flush) hold no entry
  auto q_flush = [&](bool full) {
    const bool valid = full || lane < q.n;
    const uint32_t s1[1] = {valid ? (q.e0 & 0xFFFFu) : kIplNoSlot};
    const uint32_t d1[1] = {valid ? (q.e0 >> 16) : kIplNoSlot};
    const uint32_t b1[1] = {kDropQ ? q.e1 & kQBytes : q.e1};
    const uint32_t m1[1] = {kDropQ ? (kVerdictDropped << 8) | ((q.e1 >> 29) << 18) : q.e2};
    l4_records<NG, SIG, 1, 2>(G, l4, ds, b1, m1, s1, d1);
  };
  const uint64_t start = (uint64_t)blockIdx.x * a.chunk;
  const uint64_t end = start + a.chunk < a.n ? start + a.chunk : a.n;
  uint64_t tail = start;
  if (kVec && start + 4 <= end) {
    // 4 records per thread per step; the next step's 64 bytes are loaded before this
    // step's probes and updates run, so HBM reads stay in flight during the LDS work
    const uint64_t v0 = start >> 2, vn = (end - start) >> 2, vend = v0 + vn;
    const uint4 *s4 = (const uint4 *)a.c.src, *d4 = (const uint4 *)a.c.dst;
    const uint4 *b4 = (const uint4 *)a.c.bytes, *m4 = (const uint4 *)a.c.meta;
    // the loop is wave-uniform (SpillQ's cross-lane pushes need every lane present):
    // lanes past the end load a clamped vector and update nothing
    const uint64_t vwave = v0 + (threadIdx.x & ~63u);
    const uint64_t vlast = vend - 1;  // vn >= 1
    uint64_t vl = vwave + lane < vend ? vwave + lane : vlast;
    uint4 ns = rec_ld(&s4[vl]), nd = rec_ld(&d4[vl]), nbv = rec_ld(&b4[vl]), nm = rec_ld(&m4[vl]);
    for (uint64_t vw = vwave; vw < vend; vw += blockDim.x) {
      const bool act = vw + lane < vend;
      const uint4 vs = ns, vd = nd, vb = nbv, vm = nm;
      vl = vw + blockDim.x + lane < vend ? vw + blockDim.x + lane : vlast;  // clamped: no branch
      ns = rec_ld(&s4[vl]);
      nd = rec_ld(&d4[vl]);
      nbv = rec_ld(&b4[vl]);
      nm = rec_ld(&m4[vl]);
      const uint32_t ip[8] = {vs.x, vs.y, vs.z, vs.w, vd.x, vd.y, vd.z, vd.w};
      uint32_t sl[8];
      iv.lookup8(ip, act, sl);
      const uint32_t ss[4] = {sl[0], sl[1], sl[2], sl[3]}, sd[4] = {sl[4], sl[5], sl[6], sl[7]};
      const uint32_t by[4] = {vb.x, vb.y, vb.z, vb.w}, me[4] = {vm.x, vm.y, vm.z, vm.w};
      if (!G.any_spilled) {
        l4_records<NG, SIG, 4, 0>(G, l4, ds, by, me, ss, sd);
        continue;
      }
      l4_records<NG, SIG, 4, 1>(G, l4, ds, by, me, ss, sd);
      // records that update a spilled group -> SpillQ (rolled: one copy of the flush)
      uint32_t x0 = ss[0] | sd[0] << 16, x1 = ss[1] | sd[1] << 16, x2 = ss[2] | sd[2] << 16,
               x3 = ss[3] | sd[3] << 16;
      uint32_t y0 = by[0], y1 = by[1], y2 = by[2], y3 = by[3];
      uint32_t z0 = me[0], z1 = me[1], z2 = me[2], z3 = me[3];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t ver = meta_verdict(z0);
        const uint32_t fm = (G.any_flags && ver == kVerdictForwarded && meta_proto(z0) == 6)
                                ? flag_label_mask(meta_flags(z0)) : 0u;
        bool need = false;
#pragma unroll
        for (int g = 0; g < NG; ++g)
          if (G.fam[g] != FAM_COUNT && !G.inl[g]) need |= fam_hit(G.fam[g], ver, fm);
        need = need & (x0 != 0xFFFFFFFFu);  // some side is a pod
        bool full;
        if (kDropQ) {
          if (__builtin_expect(need && y0 > kQBytes, 0)) {  // jumbo bytes: straight to the bins
            const uint32_t r = meta_reason(z0), sdd = x0 >> 16, sss = x0 & 0xFFFFu;
            const uint32_t kd = G.keyed[1] ? sdd : 0u, ks = G.keyed[1] ? sss : 0u;
            if (sdd != kIplNoSlot) atomicAdd(&a.d.byt[G.base[1] + mul_u24(kd * 2u, G.nsub[1]) + r], (unsigned long long)y0);
            if (sss != kIplNoSlot) atomicAdd(&a.d.byt[G.base[1] + mul_u24(ks * 2u + 1u, G.nsub[1]) + r], (unsigned long long)y0);
          }
          full = q.push2(need, lane, x0, (y0 > kQBytes ? 0u : y0) | (meta_reason(z0) << 29));
        } else {
          full = q.push(need, lane, x0, y0, z0);
        }
        if (full) {
          q_flush(true);
          q.next();
        }
        x0 = x1; x1 = x2; x2 = x3;
        y0 = y1; y1 = y2; y2 = y3;
        z0 = z1; z1 = z2; z2 = z3;
      }
    }
    tail = start + (vn << 2);
  }
  for (uint64_t i = tail + threadIdx.x; i < end; i += blockDim.x) {
    const uint32_t ss[1] = {iv.lookup(a.c.src[i])};
    const uint32_t sd[1] = {iv.lookup(a.c.dst[i])};
    const uint32_t by[1] = {a.c.bytes[i]}, me[1] = {a.c.meta[i]};
    l4_records<NG, SIG, 1>(G, l4, ds, by, me, ss, sd);
  }
  if (G.any_spilled && q.n) q_flush(false);

  __syncthreads();
  if (a.stage_a) {
    // staged flush: plain 16-byte stores of this workgroup's bins; stage_reduce_kernel
    // sums the copies (a global atomic per bin per workgroup costs more)
    uint4 *dst = (uint4 *)(a.stage_a + (size_t)blockIdx.x * a.stage_a_stride);
    for (uint32_t i = threadIdx.x; i < a.stage_a_stride / 4; i += blockDim.x) dst[i] = ((const uint4 *)bins)[i];
  } else {
    // flush group by group (each LDS group is contiguous): 256-byte contiguous atomics
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (G.fam[g] == FAM_COUNT || !G.inl[g]) continue;
      const bool with_bytes = G.fam[g] <= FAM_DROP;
      const uint32_t hi = G.base[g] + a.p.g[g].nbins;
      for (uint32_t i = G.base[g] + threadIdx.x; i < hi; i += blockDim.x) {
        const uint32_t w = bins[i];
        if (!w) continue;
        if (with_bytes) {
          atomicAdd(&a.d.cnt[i], (unsigned long long)(w >> kL4CountShift));
          const uint32_t by = w & kL4BytesMask;
          if (by) atomicAdd(&a.d.byt[i], (unsigned long long)by);
        } else {
          atomicAdd(&a.d.cnt[i], (unsigned long long)w);
        }
      }
    }
  }
  spill_counts_out(a, bins + L4 + 64);
}

// ---- sketch pass (config C3): count-min by window partition, HLL direct -------------
// Count-min updates are 4 random u32 adds per record into d x 2^w counters (16 MiB at
// C3): as global atomics they run at the memory-side atomic rate (one 64-B request per
// lane), ~40x slower than streaming.  Instead sketch_scatter_kernel appends each update's
// column offset (u16) to a per-(workgroup, window) list -- a window is 2^15 columns of
// one row -- with one LDS counter per window, and cms_fold_kernel adds one window's
// lists into LDS and then into the row with coalesced 256-byte atomics.  Exact: an
// update whose list is full falls back to its global atomic.
struct SketchK {
  const uint32_t *src, *dst, *ports, *meta;
  uint64_t n, chunk;
  DevIpTable t;
  uint32_t *cms;
  uint32_t depth, wlog2, wshift, nwin, cap;  // nwin = 0: every update is a global atomic
  uint16_t *lists;   // [gridDim.x][nwin][cap]
  uint32_t *counts;  // [gridDim.x][nwin]
  uint32_t *hll;
  uint32_t p;
  // HLL updates bucketed in two levels: the scatter appends to the list of the source
  // pod's super-window (2^hsshift pods, few lists, so L2 keeps them whole-line), the
  // split pass re-buckets each super-window into fine windows (2^hshift pods, <= 128 KiB
  // of registers), the fold applies a fine window in LDS.  u32 entry:
  // pod-in-super-window << (p + 6) | register << 6 | rank.  hnsup = 0: direct CAS.
  uint32_t hshift, hsshift, hnsup, hnwin, hcap;
  uint32_t *hlists;   // level 1: [gridDim.x][hnsup][hcap]
  uint32_t *hcounts;  // [gridDim.x][hnsup]
  uint32_t hb2, hcap2;  // split workgroups per super-window, level-2 list capacity
  uint32_t *hlists2;  // level 2: [hnsup][hb2][2^(hsshift - hshift)][hcap2]
  uint32_t *hcounts2; // [hnsup][hb2][2^(hsshift - hshift)]
  uint32_t hll_slots; // slots covered by the registers
  const uint8_t *ipl; // LDS image of every pod IP (source lookups), or null: HBM table
  uint32_t ipl_nb, ipl_seed, ipl_bytes;
  uint32_t ipl_npfx, ipl_pfx[kIprMaxPfx];  // radix image (sketch_stage_kernel<2 / 3, .>)
  uint32_t ipl_dr[kIprMaxPfx];             // dense radix descriptors (<3, .>)
  // LDS staging of list appends (sketch_stage_kernel): per count-min window sbc u16 and
  // per HLL super-window sbh u32 entries (powers of two), flushed every `round` records
  // per lane (2 or 4) as contiguous runs
  uint32_t sbc, sbh, round;
  uint32_t sbs;  // hll_split_kernel staging ring per fine window (0: unstaged)
  uint32_t sbs_every;  // hll_split_kernel: rounds between flushes of the rings
  // deferred folds: the scatter appends after the fill earlier launches stored in
  // counts / hcounts (their lists are folded later, once, by the fold kernels)
  uint32_t accum;
};

// Walks n4 16-byte list words starting at lane t with stride `stride`, four loads in
// flight per lane before the updates (fold kernels are latency-bound on list reads).
template <class F>
__device__ __forceinline__ void walk_u4(const uint4 *e4, uint32_t n4, uint32_t t, uint32_t stride, F &&f) {
  uint32_t j = t;
  for (; j + 3 * stride < n4; j += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = e4[j + q * stride];
#pragma unroll
    for (int q = 0; q < 4; ++q) f(v[q]);
  }
  for (; j < n4; j += stride) f(e4[j]);
}

// One record's sketch updates: each count-min row's column is appended to the list of
// its window (row, column >> wshift) and each HLL (pod, register, rank) to the list of
// its pod window; a full list falls back to the global atomic (exact, slow).
struct SketchLists {
  const SketchK &k;
  uint32_t *wcnt, *hcnt;
  uint16_t *mine;
  uint32_t *hmine;
  uint32_t wmask, hi_bits, omask;
  __device__ __forceinline__ void record(uint32_t s, uint32_t d, uint32_t ports, uint32_t meta,
                                         const Lk &ls) const {
    if (k.depth) {
      const uint64_t base = cms_base(s, d, ports, meta_proto(meta));
#pragma unroll 4
      for (uint32_t r = 0; r < k.depth; ++r) {
        const uint32_t col = cms_col(base, r, wmask);
        bool direct = k.nwin == 0;
        if (!direct) {
          const uint32_t w = (r << hi_bits) | (col >> k.wshift);
          const uint32_t pos = atomicAdd(&wcnt[w], 1u);
          direct = pos >= k.cap;
          if (!direct) mine[(size_t)w * k.cap + pos] = (uint16_t)(col & omask);
        }
        if (direct) atomicAdd(&k.cms[((size_t)r << k.wlog2) + col], 1u);
      }
    }
    if (k.p && ls.slot >= 0 && (uint32_t)ls.slot < k.hll_slots) {
      bool direct = k.hnsup == 0;
      if (!direct) {
        const uint64_t h = hll_hash(d);
        const uint32_t idx = (uint32_t)(h >> (64 - k.p));
        const uint32_t rho = (uint32_t)__builtin_clzll((h << k.p) | (1ULL << (k.p - 1))) + 1u;
        const uint32_t w = (uint32_t)ls.slot >> k.hsshift;
        const uint32_t pos = atomicAdd(&hcnt[w], 1u);
        direct = pos >= k.hcap;
        if (!direct)
          hmine[(size_t)w * k.hcap + pos] =
              (((uint32_t)ls.slot & ((1u << k.hsshift) - 1u)) << (k.p + 6)) | (idx << 6) | rho;
      }
      if (direct) hll_update(k.hll, k.p, ls.slot, d);
    }
  }
};

// Sketch pass over the records.  kVec: 4 consecutive records per lane per step (16-byte
// loads per column) and the 8 IP-table probes of their 4 sources issued back to back, so
// a wave keeps ~12 loads in flight instead of waiting on one record's probe at a time.
template <bool kVec, bool kLdsIp>
__global__ __launch_bounds__(1024) void sketch_scatter_kernel(SketchK k) {
  // [nwin] count-min list fill counters, then [hnwin] HLL list fill counters, then
  // (kLdsIp) the IP image at the next 16-byte boundary
  extern __shared__ __attribute__((aligned(16))) uint32_t wcnt[];
  uint32_t *hcnt = wcnt + k.nwin;
  const uint32_t img_off = (k.nwin + k.hnsup + 3u) & ~3u;
  const uint32_t *keys = wcnt + img_off;
  const uint16_t *vals = (const uint16_t *)((const uint8_t *)keys + ipl_vals_offset(k.ipl_nb));
  for (uint32_t i = threadIdx.x; i < k.nwin + k.hnsup; i += blockDim.x)
    wcnt[i] = !k.accum ? 0u
              : i < k.nwin ? k.counts[(size_t)blockIdx.x * k.nwin + i]
                           : k.hcounts[(size_t)blockIdx.x * k.hnsup + (i - k.nwin)];
  if (kLdsIp)
    for (uint32_t i = threadIdx.x; i < k.ipl_bytes / 16; i += blockDim.x)
      ((uint4 *)(wcnt + img_off))[i] = ((const uint4 *)k.ipl)[i];
  __syncthreads();
  auto lds_lookup = [&](uint32_t ip) {
    const uint32_t v = vals[ipl_probe_index(keys, k.ipl_nb, k.ipl_seed, ip)];
    return Lk{v == kIplNoSlot ? -1 : (int32_t)v, 0u};
  };
  const uint64_t start = (uint64_t)blockIdx.x * k.chunk;
  const uint64_t end = start + k.chunk < k.n ? start + k.chunk : k.n;
  const SketchLists L{k, wcnt, hcnt, k.lists + (size_t)blockIdx.x * k.nwin * k.cap,
                      k.hlists + (size_t)blockIdx.x * k.hnsup * k.hcap, (1u << k.wlog2) - 1u,
                      k.wlog2 - k.wshift, (1u << k.wshift) - 1u};
  const bool need_ports = k.depth != 0 && k.ports;
  const Lk none{-1, 0};
  uint64_t tail = start;
  if (kVec && start + 4 <= end) {
    const uint64_t v0 = start >> 2, vend = v0 + ((end - start) >> 2);
    const uint4 *s4 = (const uint4 *)k.src, *d4 = (const uint4 *)k.dst;
    const uint4 *p4 = (const uint4 *)k.ports, *m4 = (const uint4 *)k.meta;
    // software pipeline: the next step's record loads are in flight while this step's
    // probes and list appends run
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    uint64_t v = v0 + threadIdx.x;
    uint4 ns = z4, nd = z4, nm = z4, np = z4;
    if (v < vend) {
      ns = s4[v];
      nd = d4[v];
      nm = m4[v];
      np = need_ports ? p4[v] : z4;
    }
    for (; v < vend; v += blockDim.x) {
      const uint4 vs = ns, vd = nd, vm = nm, vp = np;
      const uint64_t vn = v + blockDim.x;
      if (vn < vend) {
        ns = s4[vn];
        nd = d4[vn];
        nm = m4[vn];
        np = need_ports ? p4[vn] : z4;
      }
      Lk ls[4] = {none, none, none, none};
      if (kLdsIp) {
        ls[0] = lds_lookup(vs.x);
        ls[1] = lds_lookup(vs.y);
        ls[2] = lds_lookup(vs.z);
        ls[3] = lds_lookup(vs.w);
      } else if (k.p) {
        const uint32_t ip[4] = {vs.x, vs.y, vs.z, vs.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) ls[j] = ip_lookup(k.t, ip[j]);
      }
      L.record(vs.x, vd.x, vp.x, vm.x, ls[0]);
      L.record(vs.y, vd.y, vp.y, vm.y, ls[1]);
      L.record(vs.z, vd.z, vp.z, vm.z, ls[2]);
      L.record(vs.w, vd.w, vp.w, vm.w, ls[3]);
    }
    tail = start + ((end - start) & ~3ULL);
  }
  for (uint64_t i = tail + threadIdx.x; i < end; i += blockDim.x) {
    const uint32_t s = k.src[i];
    L.record(s, k.dst[i], need_ports ? k.ports[i] : 0u, k.meta[i],
             kLdsIp ? lds_lookup(s) : k.p ? ip_lookup(k.t, s) : none);
  }
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < k.nwin; w += blockDim.x)
    k.counts[(size_t)blockIdx.x * k.nwin + w] = wcnt[w] < k.cap ? wcnt[w] : k.cap;
  for (uint32_t w = threadIdx.x; w < k.hnsup; w += blockDim.x)
    k.hcounts[(size_t)blockIdx.x * k.hnsup + w] = hcnt[w] < k.hcap ? hcnt[w] : k.hcap;
}

// Staged scatter (the default when LDS allows): appends land in per-window LDS staging
// rings and are written out as contiguous runs once per round, so every list write is a
// coalesced wave store instead of one L2 request per 2- or 4-byte entry (PMC on the
// unstaged kernel: 45 B written per record for 12 B of list entries).
//
// Per-round counters: rc[w] counts window w's appends of this round (reset by the flush)
// and rb[w] is the list length at the round's start, so an append's ring slot is the
// value its LDS atomic returns -- one LDS round trip per update, no read of rb.  Every
// update of a record (kD count-min rows and the HLL entry) is computed first and the
// atomics of two records are issued back to back, so 2 x (kD + 1) LDS round trips are in
// flight per lane instead of one after another.  A position past the ring (rare: rings
// hold 1.5 x a round's mean + 64) is stored straight into the list at rb + pos; a list
// position past the capacity falls back to the global atomic (exact).
// kIp: source lookup 0 HBM table, 1 LDS cuckoo image, 2 LDS radix image, 3 LDS dense radix
// image.
// kD: count-min depth fixed at compile time (4), or 0 = k.depth.
__host__ __device__ inline uint32_t stage_words(uint32_t nwin, uint32_t hnsup, uint32_t sbc, uint32_t sbh) {
  // rc, rb per window + hc, hb per super-window; u16 rings (+ one dummy u32); u32 rings
  // (+ 64 dummies)
  return ((2u * (nwin + hnsup) + 3u) & ~3u) + ((nwin * sbc / 2u + 1u + 3u) & ~3u) + hnsup * sbh + 64u;
}

template <int kIp, int kD>
__global__ __launch_bounds__(1024) void sketch_stage_kernel(SketchK k) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  const uint32_t nw = k.nwin, nh = k.hnsup, sbc = k.sbc, sbh = k.sbh;
  uint32_t *rc = sm, *rb = sm + nw, *hc = rb + nw, *hb = hc + nh;
  uint16_t *cst = (uint16_t *)(sm + ((2u * (nw + nh) + 3u) & ~3u));
  const uint32_t cdummy = nw * sbc;  // u16 index of the rings' dummy entry
  uint32_t *hst = (uint32_t *)cst + ((nw * sbc / 2u + 1u + 3u) & ~3u);
  const uint32_t hdummy = nh * sbh;  // 64 u32 dummies follow the HLL rings
  const uint32_t img_off = stage_words(nw, nh, sbc, sbh);
  const uint8_t *img = (const uint8_t *)(sm + img_off);
  // rc / hc (this round's appends) start at 0; rb / hb (list fill) at 0, or with deferred
  // folds at the fill the previous launches stored
  for (uint32_t i = threadIdx.x; i < 2u * (nw + nh); i += blockDim.x) {
    uint32_t v = 0u;
    if (k.accum && i >= nw && i < 2u * nw) v = k.counts[(size_t)blockIdx.x * nw + (i - nw)];
    if (k.accum && i >= 2u * nw + nh) v = k.hcounts[(size_t)blockIdx.x * nh + (i - 2u * nw - nh)];
    sm[i] = v;
  }
  if (kIp) fill_lds_u4((uint4 *)(sm + img_off), (const uint4 *)k.ipl, k.ipl_bytes / 16);
  __syncthreads();
  const uint32_t D = kD ? (uint32_t)kD : k.depth;
  const uint32_t wmask = (1u << k.wlog2) - 1u, hi_bits = k.wlog2 - k.wshift, omask = (1u << k.wshift) - 1u;
  const uint32_t lane = threadIdx.x & 63u;
  uint16_t *mine = k.lists + (size_t)blockIdx.x * nw * k.cap;
  uint32_t *hmine = k.hlists + (size_t)blockIdx.x * nh * k.hcap;
  // kIp 1 / 2 / 3: the cuckoo / radix / dense radix image (IplView kinds 0 / 1 / 2)
  const IplView<kIp == 3 ? 2 : kIp == 2 ? 1 : 0> iv{img,          k.ipl_nb,     k.ipl_seed,   k.ipl_npfx,
                                                    k.ipl_pfx[0], k.ipl_pfx[1], k.ipl_pfx[2], k.ipl_pfx[3],
                                                    k.ipl_dr[0],  k.ipl_dr[1],  k.ipl_dr[2],  k.ipl_dr[3]};
  auto src_slot = [&](uint32_t ip) -> uint32_t {  // slot or >= hll_slots
    if (kIp) return iv.lookup(ip);
    const Lk l = k.p ? ip_lookup(k.t, ip) : Lk{-1, 0};
    return l.slot < 0 ? 0xFFFFFFFFu : (uint32_t)l.slot;
  };
  // count-min entry that cannot be staged or listed: the global atomic
  auto cms_direct = [&](uint32_t w, uint32_t e) {
    const uint32_t r = w >> hi_bits, col = ((w & ((1u << hi_bits) - 1u)) << k.wshift) | e;
    atomicAdd(&k.cms[((size_t)r << k.wlog2) + col], 1u);
  };
  auto hll_direct = [&](uint32_t wh, uint32_t e) {
    const uint32_t slot = (wh << k.hsshift) | (e >> (k.p + 6));
    const size_t byte = ((size_t)slot << k.p) + ((e >> 6) & ((1u << k.p) - 1u));
    const uint32_t rho = e & 63u, sh = (uint32_t)(byte & 3) * 8u;
    uint32_t *word = k.hll + (byte >> 2);
    uint32_t old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (((old >> sh) & 0xFFu) < rho) {
      const uint32_t prev = atomicCAS(word, old, (old & ~(0xFFu << sh)) | (rho << sh));
      if (prev == old) break;
      old = prev;
    }
  };
  // R records of this lane (act: real records) through every update: all positions
  // reserved first, then the ring stores (dummy entries absorb the rest), then the rare
  // overflow path for the whole wave at once
  constexpr int kMaxD = kD ? kD : 8;
  auto records = [&](auto R, const uint32_t *s, const uint32_t *d, const uint32_t *pt, const uint32_t *mt,
                     const bool *act) {
    constexpr int NR = decltype(R)::value;
    uint32_t we[NR][kMaxD], pos[NR][kMaxD], he[NR], hw[NR], hp[NR];
    bool hv[NR];
    uint32_t sl[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) sl[j] = k.p ? src_slot(s[j]) : 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      if (D) {
        const uint64_t base = cms_base(s[j], d[j], pt[j], meta_proto(mt[j]));
#pragma unroll
        for (int r = 0; r < kMaxD; ++r) {
          if (!kD && (uint32_t)r >= D) break;
          const uint32_t col = cms_col(base, (uint32_t)r, wmask);
          we[j][r] = ((((uint32_t)r << hi_bits) | (col >> k.wshift)) << 16) | (col & omask);
        }
      }
      hv[j] = act[j] && k.p && sl[j] < k.hll_slots;
      hw[j] = 0u;
      he[j] = 0u;
      if (k.p) {
        const uint64_t h = hll_hash(d[j]);
        const uint32_t idx = (uint32_t)(h >> (64 - k.p));
        const uint32_t rho = (uint32_t)__builtin_clzll((h << k.p) | (1ULL << (k.p - 1))) + 1u;
        hw[j] = hv[j] ? sl[j] >> k.hsshift : 0u;
        he[j] = ((sl[j] & ((1u << k.hsshift) - 1u)) << (k.p + 6)) | (idx << 6) | rho;
      }
    }
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      if (D) {
#pragma unroll
        for (int r = 0; r < kMaxD; ++r) {
          if (!kD && (uint32_t)r >= D) break;
          pos[j][r] = act[j] ? atomicAdd(&rc[we[j][r] >> 16], 1u) : 0xFFFFFFFFu;
        }
      }
      hp[j] = hv[j] ? atomicAdd(&hc[hw[j]], 1u) : 0xFFFFFFFFu;
    }
    bool slow = false;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      if (D) {
#pragma unroll
        for (int r = 0; r < kMaxD; ++r) {
          if (!kD && (uint32_t)r >= D) break;
          const uint32_t w = we[j][r] >> 16, p = pos[j][r];
          const bool ring = p < sbc;
          cst[ring ? mul_u24(w, sbc) + p : cdummy] = (uint16_t)we[j][r];  // 24-bit: full-rate multiply
          slow |= act[j] & !ring;
        }
      }
      const bool hring = hp[j] < sbh;
      hst[hring ? mul_u24(hw[j], sbh) + hp[j] : hdummy + lane] = he[j];
      slow |= hv[j] & !hring;
    }
    if (__builtin_expect(__ballot(slow) != 0, 0)) {  // past a ring: list at rb + pos, or global
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        if (D) {
#pragma unroll
          for (int r = 0; r < kMaxD; ++r) {
            if (!kD && (uint32_t)r >= D) break;
            const uint32_t w = we[j][r] >> 16, p = pos[j][r];
            if (!act[j] || p < sbc) continue;
            const uint32_t lp = rb[w] + p;
            if (lp < k.cap) mine[(size_t)w * k.cap + lp] = (uint16_t)we[j][r];
            else cms_direct(w, we[j][r] & 0xFFFFu);
          }
        }
        if (!hv[j] || hp[j] < sbh) continue;
        const uint32_t lp = hb[hw[j]] + hp[j];
        if (lp < k.hcap) hmine[(size_t)hw[j] * k.hcap + lp] = he[j];
        else hll_direct(hw[j], he[j]);
      }
    }
  };
  // all threads, between barriers: each window's staged run to its list (positions past
  // the capacity: the global atomic), then the round counters reset.  A wave takes kG
  // windows at a time and issues every LDS read of them (counters, then up to kIt ring
  // entries per lane and window) before its global stores, so a flush costs a few LDS
  // round trips per wave instead of a few per window.
  auto flush_rings = [&](auto G, auto IT, uint32_t nwin, auto *ring, uint32_t sb, uint32_t *cnt, uint32_t *bas,
                         auto *list, uint32_t cap, auto &&direct) {
    constexpr int kG = decltype(G)::value, kIt = decltype(IT)::value;
    using T = typename std::remove_pointer<decltype(list)>::type;
    const uint32_t wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    for (uint32_t w0 = wave; w0 < nwin; w0 += kG * nwaves) {
      uint32_t n[kG], b[kG];
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        const uint32_t w = w0 + q * nwaves;
        n[q] = w < nwin ? cnt[w] : 0u;
        b[q] = w < nwin ? bas[w] : 0u;
      }
      T v[kG][kIt];
#pragma unroll
      for (int q = 0; q < kG; ++q)
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
          const uint32_t p = lane + 64u * it;
          v[q][it] = p < min(n[q], sb) ? ring[mul_u24(w0 + q * nwaves, sb) + p] : (T)0;
        }
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        const uint32_t w = w0 + q * nwaves, m = min(n[q], sb);
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
          const uint32_t p = lane + 64u * it;
          if (p >= m) continue;
          if (b[q] + p < cap) list[(size_t)w * cap + b[q] + p] = v[q][it];
          else direct(w, (uint32_t)v[q][it]);
        }
        for (uint32_t p = lane + 64u * kIt; p < m; p += 64) {  // rings longer than kIt * 64
          const T e = ring[w * sb + p];
          if (b[q] + p < cap) list[(size_t)w * cap + b[q] + p] = e;
          else direct(w, (uint32_t)e);
        }
        if (lane == 0 && w < nwin) {
          bas[w] = b[q] + n[q];
          cnt[w] = 0u;
        }
      }
    }
  };
  auto flush = [&]() {
    flush_rings(std::integral_constant<int, 4>{}, std::integral_constant<int, 4>{}, nw, cst, sbc, rc, rb, mine,
                k.cap, cms_direct);
    flush_rings(std::integral_constant<int, 1>{}, std::integral_constant<int, 8>{}, nh, hst, sbh, hc, hb, hmine,
                k.hcap, hll_direct);
  };
  const uint64_t start = (uint64_t)blockIdx.x * k.chunk;
  const uint64_t end = start + k.chunk < k.n ? start + k.chunk : k.n;
  const bool need_ports = D != 0 && k.ports;
  uint64_t tail = start;
  if (start + 4 <= end) {
    const uint64_t v0 = start >> 2, vend = v0 + ((end - start) >> 2);
    const uint4 *s4 = (const uint4 *)k.src, *d4 = (const uint4 *)k.dst;
    const uint4 *p4 = (const uint4 *)k.ports, *m4 = (const uint4 *)k.meta;
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    uint4 ns = z4, nd = z4, nm = z4, np = z4;
    if (v0 + threadIdx.x < vend) {
      const uint64_t v = v0 + threadIdx.x;
      ns = rec_ld(&s4[v]);
      nd = rec_ld(&d4[v]);
      nm = rec_ld(&m4[v]);
      np = need_ports ? rec_ld(&p4[v]) : z4;
    }
    // block-uniform trip count: every thread reaches the flush barriers
    for (uint64_t vb = v0; vb < vend; vb += blockDim.x) {
      const uint64_t v = vb + threadIdx.x;
      const bool a = v < vend;
      const uint4 vs = ns, vd = nd, vm = nm, vp = np;
      const uint64_t vn = v + blockDim.x;
      if (vn < vend) {
        ns = rec_ld(&s4[vn]);
        nd = rec_ld(&d4[vn]);
        nm = rec_ld(&m4[vn]);
        np = need_ports ? rec_ld(&p4[vn]) : z4;
      }
      const bool act[2] = {a, a};
      {
        const uint32_t s[2] = {vs.x, vs.y}, d[2] = {vd.x, vd.y}, pt[2] = {vp.x, vp.y}, mt[2] = {vm.x, vm.y};
        records(std::integral_constant<int, 2>{}, s, d, pt, mt, act);
      }
      if (k.round == 2) {
        __syncthreads();
        flush();
        __syncthreads();
      }
      {
        const uint32_t s[2] = {vs.z, vs.w}, d[2] = {vd.z, vd.w}, pt[2] = {vp.z, vp.w}, mt[2] = {vm.z, vm.w};
        records(std::integral_constant<int, 2>{}, s, d, pt, mt, act);
      }
      __syncthreads();
      flush();
      __syncthreads();
    }
    tail = start + ((end - start) & ~3ULL);
  }
  // < 4 records left (the last workgroup's chunk): one more staged round
  if (tail < end) {  // block-uniform
    const uint64_t i = tail + threadIdx.x;
    const bool a = i < end;
    const uint32_t s[1] = {a ? k.src[i] : 0u}, d[1] = {a ? k.dst[i] : 0u},
                   pt[1] = {a && need_ports ? k.ports[i] : 0u}, mt[1] = {a ? k.meta[i] : 0u};
    const bool act[1] = {a};
    records(std::integral_constant<int, 1>{}, s, d, pt, mt, act);
    __syncthreads();
    flush();
    __syncthreads();
  }
  for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x)
    k.counts[(size_t)blockIdx.x * nw + w] = rb[w] < k.cap ? rb[w] : k.cap;
  for (uint32_t w = threadIdx.x; w < nh; w += blockDim.x)
    k.hcounts[(size_t)blockIdx.x * nh + w] = hb[w] < k.hcap ? hb[w] : k.hcap;
}

// HLL level 2: workgroup (super-window s, part b) reads scatter lists b, b + hb2, ... of
// super-window s and appends each entry to its fine window's list (s, b, fine window);
// a full list applies the entry with the global CAS (exact).
__global__ __launch_bounds__(1024) void hll_split_kernel(SketchK k, uint32_t n_lists) {
  // LDS: [nfine] fill counters, [nfine] flushed positions, then (k.sbs) [nfine][sbs]
  // staging rings: a round of 4096 entries is appended, then written out per fine window
  // as contiguous runs (as in sketch_stage_kernel)
  extern __shared__ __attribute__((aligned(16))) uint32_t fcnt[];
  const uint32_t s = blockIdx.x / k.hb2, b = blockIdx.x % k.hb2;
  const uint32_t fshift = k.hsshift - k.hshift, nfine = 1u << fshift;
  uint32_t *ffl = fcnt + nfine, *ring = fcnt + 2 * nfine;
  const uint32_t R = k.sbs;
  for (uint32_t i = threadIdx.x; i < 2 * nfine; i += blockDim.x) fcnt[i] = 0u;
  __syncthreads();
  const size_t base2 = ((size_t)s * k.hb2 + b) * nfine;
  uint32_t *out = k.hlists2 + base2 * k.hcap2;
  const uint32_t psh = k.p + 6, pmask = (1u << k.hsshift) - 1u;
  auto put = [&](uint32_t x) {
    const uint32_t pod = (x >> psh) & pmask, wf = pod >> k.hshift;
    const uint32_t pos = atomicAdd(&fcnt[wf], 1u);
    if (pos < k.hcap2) {
      if (R && pos - ffl[wf] < R) ring[wf * R + (pos & (R - 1u))] = x;
      else out[(size_t)wf * k.hcap2 + pos] = x;
      return;
    }
    const uint32_t slot = (s << k.hsshift) | pod;  // full list: the global CAS
    const size_t byte = ((size_t)slot << k.p) + ((x >> 6) & ((1u << k.p) - 1u));
    const uint32_t rho = x & 63u, sh = (uint32_t)(byte & 3) * 8u;
    uint32_t *word = k.hll + (byte >> 2);
    uint32_t old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (((old >> sh) & 0xFFu) < rho) {
      const uint32_t prev = atomicCAS(word, old, (old & ~(0xFFu << sh)) | (rho << sh));
      if (prev == old) break;
      old = prev;
    }
  };
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  uint32_t rounds = 0;  // block-uniform
  auto flush = [&]() {
    for (uint32_t w = wave; w < nfine; w += nwaves) {
      const uint32_t f = ffl[w], c = min(fcnt[w], k.hcap2), e = min(c, f + R);
      for (uint32_t p = f + lane; p < e; p += 64) out[(size_t)w * k.hcap2 + p] = ring[w * R + (p & (R - 1u))];
      if (lane == 0) ffl[w] = c;
    }
  };
  for (uint32_t l = b; l < n_lists; l += k.hb2) {
    const uint32_t cnt = k.hcounts[(size_t)l * k.hnsup + s];  // block-uniform
    const uint32_t *e = k.hlists + ((size_t)l * k.hnsup + s) * k.hcap;  // 16-byte aligned (hcap % 16 == 0)
    if (!R) {
      const uint32_t n4 = cnt >> 2;
      walk_u4((const uint4 *)e, n4, threadIdx.x, blockDim.x, [&](const uint4 &v) {
        put(v.x);
        put(v.y);
        put(v.z);
        put(v.w);
      });
      for (uint32_t j = (n4 << 2) + threadIdx.x; j < cnt; j += blockDim.x) put(e[j]);
      continue;
    }
    // rounds of 4 entries per thread (one 16-byte load), staged and flushed; the next
    // round's load is issued before this round's appends and flush, so the list reads
    // stay in flight across the barriers
    uint4 nxt = make_uint4(0, 0, 0, 0);
    if (4 * threadIdx.x + 4 <= cnt) nxt = *(const uint4 *)(e + 4 * threadIdx.x);
    for (uint32_t r0 = 0; r0 < cnt; r0 += 4 * blockDim.x) {
      const uint32_t j = r0 + 4 * threadIdx.x;
      const uint4 cur = nxt;
      const uint32_t jn = j + 4 * blockDim.x;
      if (jn + 4 <= cnt) nxt = *(const uint4 *)(e + jn);
      if (j + 4 <= cnt) {
        const uint4 v = cur;
        put(v.x);
        put(v.y);
        put(v.z);
        put(v.w);
      } else {
        for (uint32_t q = j; q < cnt; ++q) put(e[q]);
      }
      if (++rounds % k.sbs_every == 0) {
        __syncthreads();
        flush();
        __syncthreads();
      }
    }
  }
  __syncthreads();
  if (R) {  // what the last rounds staged
    flush();
    __syncthreads();
  }
  for (uint32_t i = threadIdx.x; i < nfine; i += blockDim.x)
    k.hcounts2[base2 + i] = fcnt[i] < k.hcap2 ? fcnt[i] : k.hcap2;
}

// Workgroup w folds HLL window w: its pods' registers (<= 128 KiB) are loaded into LDS,
// every scatter workgroup's list for the window is applied with byte-max (a 32-bit CAS on
// the register's word; one wave per list), and the registers are stored back -- one
// coalesced read and write of the register array instead of a random global CAS per record.
__global__ __launch_bounds__(1024) void hll_fold_kernel(SketchK k) {
  extern __shared__ __attribute__((aligned(16))) uint32_t regs[];
  const uint32_t w = blockIdx.x;
  const uint32_t fshift = k.hsshift - k.hshift, nfine = 1u << fshift;
  const uint32_t s = w >> fshift, wf = w & (nfine - 1u);
  const uint32_t pod0 = w << k.hshift;
  const uint32_t npods = min(1u << k.hshift, k.hll_slots - pod0);
  const size_t bytes = (size_t)npods << k.p;  // multiple of 16 (p >= 4)
  uint4 *g = (uint4 *)((uint8_t *)k.hll + ((size_t)pod0 << k.p));
  fill_lds_u4((uint4 *)regs, g, (uint32_t)(bytes / 16));
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, nwaves = blockDim.x >> 6;
  const uint32_t imask = (1u << k.p) - 1u;
  const uint32_t psh = k.p + 6, fmask = (1u << k.hshift) - 1u;
  auto apply = [&](uint32_t x) {
    const uint32_t byte = (((x >> psh) & fmask) << k.p) + ((x >> 6) & imask), rho = x & 63u;
    uint32_t *word = &regs[byte >> 2];
    const uint32_t sh = (byte & 3u) * 8u;
    uint32_t old = *word;
    while (((old >> sh) & 0xFFu) < rho) {
      const uint32_t prev = atomicCAS(word, old, (old & ~(0xFFu << sh)) | (rho << sh));
      if (prev == old) break;
      old = prev;
    }
  };
  // list (s, b, wf) of every split workgroup b: one wave per list
  for (uint32_t b = threadIdx.x >> 6; b < k.hb2; b += nwaves) {
    const size_t li = ((size_t)s * k.hb2 + b) * nfine + wf;
    const uint32_t cnt = k.hcounts2[li];
    const uint32_t *e = k.hlists2 + li * k.hcap2;  // 16-byte aligned (hcap2 % 16 == 0)
    const uint32_t n4 = cnt >> 2;
    walk_u4((const uint4 *)e, n4, lane, 64u, [&](const uint4 &v) {
      apply(v.x);
      apply(v.y);
      apply(v.z);
      apply(v.w);
    });
    for (uint32_t j = (n4 << 2) + lane; j < cnt; j += 64) apply(e[j]);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < bytes / 16; i += blockDim.x) g[i] = ((const uint4 *)regs)[i];
}

// Workgroup b folds window b % nwin over scatter workgroups [part*L/P, (part+1)*L/P).
__global__ __launch_bounds__(1024) void cms_fold_kernel(SketchK k, uint32_t n_lists) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cwin[];  // [2^wshift]
  const uint32_t W = 1u << k.wshift;
  const uint32_t w = blockIdx.x % k.nwin, part = blockIdx.x / k.nwin, nparts = gridDim.x / k.nwin;
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) cwin[i] = 0u;
  __syncthreads();
  const uint32_t l0 = (uint32_t)((uint64_t)part * n_lists / nparts);
  const uint32_t l1 = (uint32_t)((uint64_t)(part + 1) * n_lists / nparts);
  // one wave per list, four 16-byte loads in flight per lane
  const uint32_t lane = threadIdx.x & 63u, nwaves = blockDim.x >> 6;
  for (uint32_t l = l0 + (threadIdx.x >> 6); l < l1; l += nwaves) {
    const uint32_t c = k.counts[(size_t)l * k.nwin + w];
    const uint16_t *e = k.lists + ((size_t)l * k.nwin + w) * k.cap;  // 16-byte aligned (cap % 8 == 0)
    const uint32_t n8 = c >> 3;
    walk_u4((const uint4 *)e, n8, lane, 64u, [&](const uint4 &v) {
      const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        atomicAdd(&cwin[x[q] & 0xFFFFu], 1u);
        atomicAdd(&cwin[x[q] >> 16], 1u);
      }
    });
    for (uint32_t j = (n8 << 3) + lane; j < c; j += 64) atomicAdd(&cwin[e[j]], 1u);
  }
  __syncthreads();
  const uint32_t hi_bits = k.wlog2 - k.wshift;
  const uint32_t r = w >> hi_bits, colbase = (w & ((1u << hi_bits) - 1u)) << k.wshift;
  uint32_t *row = k.cms + ((size_t)r << k.wlog2) + colbase;
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) {
    const uint32_t v = cwin[i];
    if (v) atomicAdd(&row[i], v);
  }
}

hipError_t launch_sketch(const SketchArgs &a, hipStream_t st, std::string *kernels, const ForkJoin *fj) {
  const bool scatter = a.passes != kSketchFolds, folds = a.passes != kSketchScatter;
  if (a.n == 0 && scatter) return hipSuccess;
  std::string names;
  SketchK k{};
  k.src = a.cols.src_ip;
  k.dst = a.cols.dst_ip;
  k.ports = a.cols.ports;
  k.meta = a.cols.meta;
  k.n = a.n;
  k.chunk = a.chunk;
  k.t = DevIpTable{a.ip_slots, a.ip_mask, a.ip_seed, a.ip_pre, a.ip_blk, 0u, {}};
  k.cms = a.cms;
  k.depth = a.cms_depth;
  k.wlog2 = a.cms_wlog2;
  k.wshift = a.win_shift;
  k.nwin = a.nwin;
  k.cap = a.cap;
  k.lists = a.lists;
  k.counts = a.counts;
  k.hll = (uint32_t *)a.hll;
  k.p = a.hll_p;
  k.hshift = a.hll_shift;
  k.hsshift = a.hll_sshift;
  k.hnsup = a.hll_nsup;
  k.hnwin = a.hll_nwin;
  k.hcap = a.hll_cap;
  k.hlists = a.hll_lists;
  k.hcounts = a.hll_counts;
  k.hb2 = a.hll_b2;
  k.hcap2 = a.hll_cap2;
  k.hlists2 = a.hll_lists2;
  k.hcounts2 = a.hll_counts2;
  k.hll_slots = a.hll_slots;
  k.accum = a.accum ? 1u : 0u;
  hipError_t e;
  size_t scatter_lds = (size_t)((a.nwin + a.hll_nsup + 3u) & ~3u) * 4;
  // source lookups in an LDS image of the IP table when it fits next to the counters
  const bool lds_ip_any = a.ipl && a.hll_p && scatter_lds + a.ipl_bytes <= kLdsBytes;
  const bool lds_ip = lds_ip_any;  // (staged kernel: either image form)
  if (lds_ip) {
    k.ipl = a.ipl;
    k.ipl_nb = a.ipl_nb;
    k.ipl_seed = a.ipl_seed;
    k.ipl_bytes = a.ipl_bytes;
    scatter_lds += a.ipl_bytes;
  }
  // 16-byte loads need aligned columns and workgroup chunks of whole vectors
  const bool vec = a.chunk % 4 == 0 && ((uintptr_t)k.src | (uintptr_t)k.dst | (uintptr_t)k.meta |
                                        (uintptr_t)(k.ports ? k.ports : k.src)) % 16 == 0;
  // staged scatter: rings sized for a round's mean appends x 1.5 + 64 (the overflow goes
  // straight to the list), flushed every 4 records per lane, or every 2 when the 4-record
  // rings do not fit; sources looked up in the radix image when the pod IPs allow one
  bool staged = !scatter;  // a fold-only call launches no scatter
  if (scatter && vec && (!a.cms_depth || a.nwin) && (!a.hll_p || a.hll_nsup) && (a.nwin || a.hll_nsup)) {
    const int ip_kind = lds_ip ? (a.ipl_dense ? 3 : a.ipl_radix ? 2 : 1) : 0;
    if (lds_ip) {
      k.ipl_npfx = a.ipl_npfx;
      for (uint32_t j = 0; j < kIprMaxPfx; ++j) {
        k.ipl_pfx[j] = a.ipl_pfx[j];
        k.ipl_dr[j] = a.ipl_dr[j];
      }
    }
    const uint32_t img = lds_ip ? a.ipl_bytes : 0u;
    for (uint32_t round : {4u, 2u}) {
      const uint64_t per_round = 1024ull * round;
      auto ring = [](uint64_t mean) {
        uint32_t r = 64;
        while (r < mean + mean / 2 + 64) r <<= 1;
        return r;
      };
      const uint32_t sbc = a.nwin ? ring(per_round * a.cms_depth / a.nwin) : 0u;
      const uint32_t sbh = a.hll_nsup ? ring(per_round / a.hll_nsup) : 0u;
      const size_t lds = (size_t)stage_words(a.nwin, a.hll_nsup, sbc, sbh) * 4 + img;
      if (lds > kLdsBytes) continue;
      k.sbc = sbc;
      k.sbh = sbh;
      k.round = round;
      const bool d4 = a.cms_depth == 4;
      const void *fn = ip_kind == 3 ? (d4 ? (const void *)sketch_stage_kernel<3, 4> : (const void *)sketch_stage_kernel<3, 0>)
                     : ip_kind == 2 ? (d4 ? (const void *)sketch_stage_kernel<2, 4> : (const void *)sketch_stage_kernel<2, 0>)
                     : ip_kind == 1 ? (d4 ? (const void *)sketch_stage_kernel<1, 4> : (const void *)sketch_stage_kernel<1, 0>)
                                    : (d4 ? (const void *)sketch_stage_kernel<0, 4> : (const void *)sketch_stage_kernel<0, 0>);
      if ((e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) != hipSuccess) return e;
      if (ip_kind == 3 && d4) hipLaunchKernelGGL((sketch_stage_kernel<3, 4>), dim3(a.blocks), dim3(1024), lds, st, k);
      else if (ip_kind == 3) hipLaunchKernelGGL((sketch_stage_kernel<3, 0>), dim3(a.blocks), dim3(1024), lds, st, k);
      else if (ip_kind == 2 && d4) hipLaunchKernelGGL((sketch_stage_kernel<2, 4>), dim3(a.blocks), dim3(1024), lds, st, k);
      else if (ip_kind == 2) hipLaunchKernelGGL((sketch_stage_kernel<2, 0>), dim3(a.blocks), dim3(1024), lds, st, k);
      else if (ip_kind == 1 && d4) hipLaunchKernelGGL((sketch_stage_kernel<1, 4>), dim3(a.blocks), dim3(1024), lds, st, k);
      else if (ip_kind == 1) hipLaunchKernelGGL((sketch_stage_kernel<1, 0>), dim3(a.blocks), dim3(1024), lds, st, k);
      else if (d4) hipLaunchKernelGGL((sketch_stage_kernel<0, 4>), dim3(a.blocks), dim3(1024), lds, st, k);
      else hipLaunchKernelGGL((sketch_stage_kernel<0, 0>), dim3(a.blocks), dim3(1024), lds, st, k);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      names = std::string("sketch_stage_kernel<") + std::to_string(ip_kind) + ", " + (d4 ? "4" : "0") + ">";
      staged = true;
      break;
    }
  }
  if (!staged) {
  // the unstaged kernel probes the cuckoo image only: a radix image is looked up in HBM
  const bool lds_ip = lds_ip_any && !a.ipl_radix && !a.ipl_dense;
  if (!lds_ip) scatter_lds = (size_t)((a.nwin + a.hll_nsup + 3u) & ~3u) * 4;
  const void *fn = vec ? (lds_ip ? (const void *)sketch_scatter_kernel<true, true>
                                 : (const void *)sketch_scatter_kernel<true, false>)
                       : (lds_ip ? (const void *)sketch_scatter_kernel<false, true>
                                 : (const void *)sketch_scatter_kernel<false, false>);
  if (scatter_lds > 64 * 1024 &&
      (e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)scatter_lds)) != hipSuccess)
    return e;
  if (vec && lds_ip) hipLaunchKernelGGL((sketch_scatter_kernel<true, true>), dim3(a.blocks), dim3(1024), scatter_lds, st, k);
  else if (vec) hipLaunchKernelGGL((sketch_scatter_kernel<true, false>), dim3(a.blocks), dim3(1024), scatter_lds, st, k);
  else if (lds_ip) hipLaunchKernelGGL((sketch_scatter_kernel<false, true>), dim3(a.blocks), dim3(1024), scatter_lds, st, k);
  else hipLaunchKernelGGL((sketch_scatter_kernel<false, false>), dim3(a.blocks), dim3(1024), scatter_lds, st, k);
  if ((e = hipGetLastError()) != hipSuccess) return e;
    names = std::string("sketch_scatter_kernel<") + (vec ? "true" : "false") + ", " + (lds_ip ? "true" : "false") + ">";
  }  // unstaged
  if (!folds) {
    if (kernels) *kernels = names;
    return hipSuccess;
  }
  // the count-min fold beside the HLL chain when both are due (-2 % per C3 step,
  // profiles/round5/exp/r5c3f_*)
  const bool fork = fj && a.nwin && a.cms_depth && a.hll_nsup && a.hll_p;
  const hipStream_t cst = fork ? fj->st2 : st;
  if (fork) {
    if ((e = hipEventRecord(fj->fork, st)) != hipSuccess || (e = hipStreamWaitEvent(fj->st2, fj->fork, 0)) != hipSuccess)
      return e;
  }
  if (a.nwin && a.cms_depth) {
    names += names.empty() ? "cms_fold_kernel" : "+cms_fold_kernel";
    const size_t lds = (size_t)4 << a.win_shift;
    if (lds > 64 * 1024 &&
        (e = hipFuncSetAttribute((const void *)cms_fold_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds)) != hipSuccess)
      return e;
    hipLaunchKernelGGL(cms_fold_kernel, dim3(a.fold_blocks), dim3(1024), lds, cst, k, a.blocks);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (a.hll_nsup && a.hll_p) {
    names += names.empty() ? "hll_split_kernel+hll_fold_kernel" : "+hll_split_kernel+hll_fold_kernel";
    // staging rings: a round (4096 entries) over nfine windows, x 2 + 64, when they fit;
    // larger rings where LDS allows, flushed every few rounds (each flush is a barrier
    // pair for the workgroup): C3's 128 fine windows take 256-entry rings, every 3 rounds
    const uint32_t nfine = 1u << (a.hll_sshift - a.hll_shift);
    const uint32_t per_round = 2 * 4096 / nfine;  // twice the mean appends per window
    uint32_t R = 64;
    while (R < per_round + 64) R <<= 1;
    if ((size_t)(2 + R) * nfine * 4 > kLdsBytes) R = 0;
    while (R && R < 256 && (size_t)(2 + 2 * R) * nfine * 4 <= kLdsBytes) R <<= 1;
    k.sbs = R;
    k.sbs_every = R ? std::max<uint32_t>(1u, (R - 64) / std::max<uint32_t>(1u, per_round)) : 1u;
    const size_t split_lds = (size_t)(2 + R) * nfine * 4;
    if ((e = hipFuncSetAttribute((const void *)hll_split_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)split_lds)) != hipSuccess)
      return e;
    hipLaunchKernelGGL(hll_split_kernel, dim3(a.hll_nsup * a.hll_b2), dim3(1024), split_lds, st, k, a.blocks);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const size_t lds = (size_t)1 << (a.hll_p + a.hll_shift);
    if (lds > 64 * 1024 &&
        (e = hipFuncSetAttribute((const void *)hll_fold_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds)) != hipSuccess)
      return e;
    hipLaunchKernelGGL(hll_fold_kernel, dim3(a.hll_nwin), dim3(1024), lds, st, k);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (fork) {
    if ((e = hipEventRecord(fj->join, fj->st2)) != hipSuccess || (e = hipStreamWaitEvent(st, fj->join, 0)) != hipSuccess)
      return e;
  }
  if (kernels) *kernels = names;
  return hipSuccess;
}

// Sums the tier-1 workgroups' staged u32 bins: part `y` of `ny` takes 1/ny of the
// copies, so each bin gets ny global atomics instead of one per workgroup.
__device__ __forceinline__ void stage_reduce_a(const uint32_t *stage, uint32_t ncopies, uint32_t stride,
                                               uint32_t L4, const Plan &p, const DevDense &d, uint32_t bx,
                                               uint32_t y, uint32_t ny) {
  const uint32_t bin = bx * blockDim.x + threadIdx.x;
  if (bin >= L4) return;
  bool packed = false;
  for (int g = 0; g < p.ngroups; ++g)
    if (bin >= p.g[g].dense_base && bin < p.g[g].dense_base + p.g[g].nbins)
      packed = p.g[g].family <= FAM_DROP;
  const uint32_t c0 = (uint32_t)(((uint64_t)ncopies * y) / ny);
  const uint32_t c1 = (uint32_t)(((uint64_t)ncopies * (y + 1)) / ny);
  unsigned long long cnt = 0, byt = 0;
#pragma unroll 8  // 8 independent copy loads in flight per lane
  for (uint32_t c = c0; c < c1; ++c) {
    const uint32_t w = stage[(size_t)c * stride + bin];
    cnt += packed ? (w >> kL4CountShift) : w;
    byt += packed ? (w & kL4BytesMask) : 0u;
  }
  if (cnt) atomicAdd(&d.cnt[bin], cnt);
  if (byt) atomicAdd(&d.byt[bin], byt);
}

// Folds the spill lists into dense counters, one LDS window of bins per workgroup.
// List (A-workgroup l, window w) holds only window w's updates, so every entry is read
// once.  Workgroup b folds window b % nwin over partition b / nwin of the lists; with
// W = 8192 bins (64 KB of LDS) two workgroups fit a CU, and the runtime sizes the grid
// to 2 x CUs so the fold runs in a single wave of the chip.  With `stage` the window
// partial is stored whole and stage_reduce_kernel sums the partitions (with the tier-1
// copies, one launch).  Round 3 measured two alternatives slower on one box
// (profiles/round3/e3a_c2_tail.jsonl): the partials summed in this launch by each window's
// last-arriving partition (agent-scope ticket; fold 0.036 -> 0.106 ms at W = 8192), and
// smaller windows with fewer partitions each (W = 2048: main kernel 0.41 -> 0.45 ms).
__global__ __launch_bounds__(1024) void spill_window_kernel(
    const uint32_t *spill, const uint32_t *spill_count, uint32_t n_lists,
    uint32_t spill_cap, uint32_t lo0, uint64_t dense_len, uint32_t W, uint32_t nwin, DevDense d,
    unsigned long long *stage) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long win[];
  const uint32_t b = blockIdx.x;
  const uint32_t w = b % nwin;
  const uint32_t part = b / nwin;
  const uint32_t nparts = gridDim.x / nwin;
  const uint64_t lo = (uint64_t)lo0 + (uint64_t)w * W;
  const uint64_t hi = lo + W < dense_len ? lo + W : dense_len;
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) win[i] = 0ULL;
  __syncthreads();
  // fewer than 2^20 entries into this window copy: no packed field can overflow
  // (entries carry < 2^18 bytes), so plain (no-return) LDS atomics suffice; otherwise
  // the exact carrying add
  uint64_t total = 0;
  for (uint32_t l = part; l < n_lists; l += nparts) total += spill_count[(size_t)l * nwin + w];
  const bool fast = total < (1ULL << 20);
  const uint32_t off_mask = W - 1, wshift = 31u - (uint32_t)__builtin_clz(W);
  auto add = [&](uint32_t x) {
    const uint32_t off = x & off_mask;
    if (x >> 31) {  // row-mask entry (kSpillRowMask): +1 to each flagged bin of the 8-bin row
      for (uint32_t m = (x >> wshift) & 0xFFu; m; m &= m - 1) {
        const uint32_t o = off + (uint32_t)__builtin_ctz(m);
        if (fast) atomicAdd(&win[o], kLdsCountOne);
        else lds_add64_exact(&win[o], (uint32_t)lo + o, 0u, d);
      }
      return;
    }
    const uint32_t nb = x >> wshift;
    if (fast) atomicAdd(&win[off], kLdsCountOne | nb);
    else lds_add64_exact(&win[off], (uint32_t)lo + off, nb, d);
  };
  // Short lists (many windows, e.g. C5's ~220: tens of entries per list) leave most of
  // the workgroup idle and serialise on list latency, so each wave takes its own list;
  // long lists (C2's drop windows: thousands of entries) keep the workgroup-wide loop.
  const uint32_t lists_here = part < n_lists ? (n_lists - part + nparts - 1) / nparts : 0u;
  if (total < (uint64_t)lists_here * 2048u) {
    const uint32_t nwaves = blockDim.x >> 6, ln = threadIdx.x & 63u;
    for (uint32_t l = part + (threadIdx.x >> 6) * nparts; l < n_lists; l += nwaves * nparts) {
      const uint32_t cnt = spill_count[(size_t)l * nwin + w];
      const uint32_t *e = spill + ((size_t)l * nwin + w) * spill_cap;
      const uint4 *e4 = (const uint4 *)e;
      const uint32_t n4 = cnt >> 2;
      for (uint32_t j = ln; j < n4; j += 64) {
        const uint4 v = e4[j];
        add(v.x);
        add(v.y);
        add(v.z);
        add(v.w);
      }
      for (uint32_t i = (n4 << 2) + ln; i < cnt; i += 64) add(e[i]);
    }
  } else {
  for (uint32_t l = part; l < n_lists; l += nparts) {
    const uint32_t cnt = spill_count[(size_t)l * nwin + w];
    const uint32_t *e = spill + ((size_t)l * nwin + w) * spill_cap;  // 16-byte aligned (cap % 4 == 0)
    const uint4 *e4 = (const uint4 *)e;
    const uint32_t n4 = cnt >> 2;
    uint32_t j = threadIdx.x;
    for (; j + 3 * blockDim.x < n4; j += 4 * blockDim.x) {  // 16 entries per lane in flight
      uint4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = e4[j + k * blockDim.x];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        add(v[k].x);
        add(v[k].y);
        add(v[k].z);
        add(v[k].w);
      }
    }
    for (; j < n4; j += blockDim.x) {
      const uint4 v = e4[j];
      add(v.x);
      add(v.y);
      add(v.z);
      add(v.w);
    }
    for (uint32_t i = (n4 << 2) + threadIdx.x; i < cnt; i += blockDim.x) add(e[i]);
  }
  }  // long lists
  __syncthreads();
  if (stage) {  // staged: this window partial, whole, for stage_reduce_kernel
    uint4 *dst = (uint4 *)(stage + ((size_t)b * W));
    for (uint32_t i = threadIdx.x; i < W / 2; i += blockDim.x) dst[i] = ((const uint4 *)win)[i];
    return;
  }
  for (uint32_t i = threadIdx.x; i < hi - lo; i += blockDim.x) {
    const unsigned long long v = win[i];
    if (v) {
      atomicAdd(&d.cnt[lo + i], v >> kLdsCountShift);
      const unsigned long long by = v & kLdsBytesMask;
      if (by) atomicAdd(&d.byt[lo + i], by);
    }
  }
}

// Sums the fold partials of every partition of a window (layout of spill_window_kernel).
__device__ __forceinline__ void stage_reduce_b(const unsigned long long *stage, uint32_t nwin, uint32_t nparts,
                                               uint32_t W, uint32_t lo0, uint64_t dense_len, const DevDense &d,
                                               uint32_t bx) {
  const uint32_t off = bx * 256u + threadIdx.x;  // over nwin * W bins
  const uint32_t w = off / W, i = off % W;
  if (w >= nwin || lo0 + (uint64_t)off >= dense_len) return;
  unsigned long long cnt = 0, byt = 0;
#pragma unroll 8  // independent partial loads in flight per lane
  for (uint32_t part = 0; part < nparts; ++part) {
    const uint32_t b = part * nwin + w;  // inverse of the fold map
    const unsigned long long v = stage[(size_t)b * W + i];
    cnt += v >> kLdsCountShift;
    byt += v & kLdsBytesMask;
  }
  if (cnt) atomicAdd(&d.cnt[lo0 + off], cnt);
  if (byt) atomicAdd(&d.byt[lo0 + off], byt);
}

// Both staged reductions in one launch (they are independent: the tier-1 bins and the
// fold partials of the spilled groups), so the step ends with one small launch instead of
// two.  Blocks [0, na) sum the tier-1 copies (na = bin blocks x ny copy parts), the rest
// the fold partials.
__global__ __launch_bounds__(256) void stage_reduce_kernel(const uint32_t *stage_a, uint32_t ncopies, uint32_t stride,
                                                           uint32_t L4, uint32_t na_x, uint32_t ny, Plan p,
                                                           const unsigned long long *stage_b, uint32_t nwin,
                                                           uint32_t nparts, uint32_t W, uint32_t lo0,
                                                           uint64_t dense_len, DevDense d) {
  const uint32_t na = stage_a ? na_x * ny : 0u;
  if (blockIdx.x < na) stage_reduce_a(stage_a, ncopies, stride, L4, p, d, blockIdx.x % na_x, blockIdx.x / na_x, ny);
  else stage_reduce_b(stage_b, nwin, nparts, W, lo0, dense_len, d, blockIdx.x - na);
}

// Writes every slot whole (k0 k1 = 0, k2 = pending, cnt byt = 0), no separate memset.
__global__ void sparse_init_kernel(unsigned long long *k0, size_t n) {
  static_assert(kSparseSlotWords == 5, "k0 k1 k2 cnt byt");
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n * kSparseSlotWords;
       i += (size_t)gridDim.x * blockDim.x)
    k0[i] = i % kSparseSlotWords == 2 ? kKeyPending : 0ULL;
}

__global__ void sparse_export_kernel(DevSparse s, size_t cap_slots, unsigned long long *out,
                                     size_t out_cap, unsigned long long *counter) {
  if (s.compact) {  // (key, count) slots, exported in the wide entry format
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < cap_slots;
         i += (size_t)gridDim.x * blockDim.x) {
      const unsigned long long key = s.k0[2 * i];
      if (!key) continue;
      const unsigned long long pos = atomicAdd(counter, 1ULL);
      if (pos >= out_cap) continue;
      unsigned long long *o = out + pos * kSparseEntryWords;
      o[0] = key & 0xFFFFFFFF00000000ULL;
      o[1] = 0ULL;
      o[2] = key & 0xFFFFFFFFULL;
      o[3] = s.k0[2 * i + 1];
      o[4] = 0ULL;
    }
    return;
  }
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < cap_slots;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t q = i * kSparseSlotWords;
    const unsigned long long k0 = s.k0[q];
    if (!k0) continue;
    const unsigned long long pos = atomicAdd(counter, 1ULL);
    if (pos >= out_cap) continue;
    unsigned long long *o = out + pos * kSparseEntryWords;
    o[0] = k0;
    o[1] = s.k1[q];
    o[2] = s.k2[q];
    o[3] = s.cnt[q];
    o[4] = s.byt[q];
  }
}

__global__ void sparse_import_kernel(DevSparse s, const unsigned long long *in, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const unsigned long long *e = in + i * kSparseEntryWords;
    sparse_add(s, e[0], e[1], e[2], e[3], e[4]);
  }
}

// ---- slot retirement and the single-process multi-GPU merge ----------------------------
// Zeroes the dense bins of retired slots: workgroup b takes dead slot b, its lanes the
// (group, side, sub) bins of that slot in every endpoint-keyed dense group.
__global__ void zero_slots_kernel(unsigned long long *cnt, unsigned long long *byt, const uint32_t *dead,
                                  Plan p) {
  const uint32_t slot = dead[blockIdx.x];
  for (int g = 0; g < p.ngroups; ++g) {
    const GroupPlan gp = p.g[g];
    if (gp.sparse || !gp.key_mode) continue;
    const uint64_t lo = gp.dense_base + (uint64_t)slot * 2u * gp.nsub;
    for (uint32_t i = threadIdx.x; i < 2u * gp.nsub; i += blockDim.x) {
      cnt[lo + i] = 0ULL;
      byt[lo + i] = 0ULL;
    }
  }
}

// Zeroes the 2^p HLL registers of each retired slot (16-byte stores).
__global__ void zero_hll_rows_kernel(uint8_t *hll, const uint32_t *dead, uint32_t p) {
  uint4 *row = (uint4 *)(hll + ((size_t)dead[blockIdx.x] << p));
  for (uint32_t i = threadIdx.x; i < (1u << p) / 16u; i += blockDim.x) row[i] = make_uint4(0, 0, 0, 0);
}

// dst[i] op= src[i] for the merge (grid-stride, vectorised where the type allows).
__global__ void add_u64_kernel(unsigned long long *dst, const unsigned long long *src, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] += src[i];
}
__global__ void add_u32_kernel(uint32_t *dst, const uint32_t *src, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] += src[i];
}
__global__ void max_u8_kernel(uint8_t *dst, const uint8_t *src, size_t n) {
  // u8 registers, 4 per lane-word: byte-wise max on the whole words, tail bytewise
  const size_t nw = n / 4;
  uint32_t *dw = (uint32_t *)dst;
  const uint32_t *sw = (const uint32_t *)src;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nw; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t a = dw[i], b = sw[i];
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = (a >> (8 * k)) & 0xFFu, y = (b >> (8 * k)) & 0xFFu;
      r |= (x > y ? x : y) << (8 * k);
    }
    dw[i] = r;
  }
  for (size_t i = nw * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = dst[i] > src[i] ? dst[i] : src[i];
}

hipError_t launch_zero_slots(uint64_t *cnt, uint64_t *byt, uint8_t *hll, uint32_t hll_p, const uint32_t *dead,
                             uint32_t ndead, const Plan &p, hipStream_t st) {
  if (!ndead) return hipSuccess;
  if (cnt) {
    hipLaunchKernelGGL(zero_slots_kernel, dim3(ndead), dim3(64), 0, st, (unsigned long long *)cnt,
                       (unsigned long long *)byt, dead, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (hll) hipLaunchKernelGGL(zero_hll_rows_kernel, dim3(ndead), dim3(256), 0, st, hll, dead, hll_p);
  return hipGetLastError();
}

hipError_t launch_merge_add_u64(uint64_t *dst, const uint64_t *src, size_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(add_u64_kernel, dim3(2048), dim3(256), 0, st, (unsigned long long *)dst,
                     (const unsigned long long *)src, n);
  return hipGetLastError();
}
hipError_t launch_merge_add_u32(uint32_t *dst, const uint32_t *src, size_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(add_u32_kernel, dim3(2048), dim3(256), 0, st, dst, src, n);
  return hipGetLastError();
}
hipError_t launch_merge_max_u8(uint8_t *dst, const uint8_t *src, size_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(max_u8_kernel, dim3(2048), dim3(256), 0, st, dst, src, n);
  return hipGetLastError();
}

// ---- enriched-flow emission (standard mode) ----------------------------------------
// Enricher.enrich (enricher.go:102-135) fills flow.Source / flow.Destination from
// Cache.GetObjByIP and exports every IPv4 flow to the output ring (export, :137-140).
// IPv4 addresses of u32 records are never "", so every record is exported; the endpoint
// is the pod's slot (its namespace/name key names the cache object whose labels and
// owner references getEndpoint copies) or -1 when GetObjByIP returns no pod (service,
// node or unknown IP: getEndpoint returns nil, :157-164).  The HBM IP table is the one
// the aggregation kernels probe.  HBM-bound: 8 B read + 8 B written per record.
__global__ __launch_bounds__(256) void enrich_kernel(DevIpTable t, const uint32_t *src, const uint32_t *dst,
                                                     uint64_t n, int32_t *os, int32_t *od, uint32_t vec) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t tail = 0;
  if (vec) {  // 4 records per lane: one 16-byte load per input column, one store per output
    const uint64_t n4 = n >> 2;
    for (uint64_t i = t0; i < n4; i += stride) {
      const uint4 s = ((const uint4 *)src)[i], d = ((const uint4 *)dst)[i];
      const Lk a0 = ip_lookup(t, s.x), a1 = ip_lookup(t, s.y), a2 = ip_lookup(t, s.z), a3 = ip_lookup(t, s.w);
      const Lk b0 = ip_lookup(t, d.x), b1 = ip_lookup(t, d.y), b2 = ip_lookup(t, d.z), b3 = ip_lookup(t, d.w);
      ((int4 *)os)[i] = make_int4(a0.slot, a1.slot, a2.slot, a3.slot);
      ((int4 *)od)[i] = make_int4(b0.slot, b1.slot, b2.slot, b3.slot);
    }
    tail = n4 << 2;
  }
  for (uint64_t i = tail + t0; i < n; i += stride) {
    os[i] = ip_lookup(t, src[i]).slot;
    od[i] = ip_lookup(t, dst[i]).slot;
  }
}

// ---- launch wrappers called by the host runtime ---------------------------------------

static DevSparse dev_sparse(const SparseView &v) {
  return DevSparse{(unsigned long long *)v.k0, (unsigned long long *)v.k1,
                   (unsigned long long *)v.k2, (unsigned long long *)v.cnt,
                   (unsigned long long *)v.byt, v.mask, (unsigned long long *)v.dropped, v.compact,
                   v.seg_log2, nullptr, nullptr, 0u, nullptr, 0u, nullptr, 0u, v.narrow};
}

template <class K>
static hipError_t launch_k(K kern, const KArgs &k, uint32_t blocks, uint32_t threads, size_t lds,
                           hipStream_t st) {
  hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)kLdsBytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, st, k);
  return hipGetLastError();
}

// dense_lds_kernel<NG, ., SIG, .> by the launch's vector loads and LDS image form
template <int NG, uint32_t SIG>
static hipError_t launch_lds(const LaunchArgs &a, const KArgs &k, uint32_t B, uint32_t T, size_t lds, hipStream_t st) {
  if (a.vec)
    return a.ipl_dense   ? launch_k(dense_lds_kernel<NG, true, SIG, 2>, k, B, T, lds, st)
           : a.ipl_radix ? launch_k(dense_lds_kernel<NG, true, SIG, 1>, k, B, T, lds, st)
                         : launch_k(dense_lds_kernel<NG, true, SIG, 0>, k, B, T, lds, st);
  return a.ipl_dense   ? launch_k(dense_lds_kernel<NG, false, SIG, 2>, k, B, T, lds, st)
         : a.ipl_radix ? launch_k(dense_lds_kernel<NG, false, SIG, 1>, k, B, T, lds, st)
                       : launch_k(dense_lds_kernel<NG, false, SIG, 0>, k, B, T, lds, st);
}

hipError_t launch_aggregate(const LaunchArgs &a, hipStream_t st, hipEvent_t between, const char **kernel) {
  if (a.n == 0) return hipSuccess;
  KArgs k{};
  k.c = DevCols{a.cols.src_ip, a.cols.dst_ip, a.cols.bytes, a.cols.meta, a.cols.ports, a.cols.dns_id};
  k.n = a.n;
  k.chunk = a.chunk;
  k.t = DevIpTable{a.ip_slots, a.ip_mask, a.ip_seed, a.ip_pre, a.ip_blk, a.ip_rpn, {}};
  for (uint32_t j = 0; j < kRadixSmall / 2; ++j) k.t.rp[j] = a.ip_rp[j];
  k.d = DevDense{(unsigned long long *)a.dense_cnt, (unsigned long long *)a.dense_byt};
  k.s = dev_sparse(a.sparse);
  k.sk = DevSketch{a.cms, a.cms_depth, a.cms_wlog2, (uint32_t *)a.hll, a.hll_p};
  k.lds_bins = a.lds_bins;
  k.spill = a.spill;
  k.spill_cap = a.spill_cap;
  k.nwin = a.nwin;
  k.win_shift = a.win_shift;
  k.spill_lo = a.spill_lo;
  k.spill_count = a.spill_count;
  k.ipl = a.ipl;
  k.ipl_nb = a.ipl_nb;
  k.ipl_seed = a.ipl_seed;
  k.ipl_bytes = a.ipl_bytes;
  k.ipl_npfx = a.ipl_npfx;
  for (uint32_t j = 0; j < kIprMaxPfx; ++j) {
    k.ipl_pfx[j] = a.ipl_pfx[j];
    k.ipl_dr[j] = a.ipl_dr[j];
  }
  k.stage_a = a.stage_a;
  k.stage_a_stride = a.stage_a_stride;
  k.stage_accum = a.stage_a && a.stage_accum ? 1u : 0u;
  k.sp_lists = (unsigned long long *)a.sp_lists;
  k.sp_counts = a.sp_counts;
  k.sp_nwin = a.sp_lists ? a.sp_nwin : 0u;
  k.sp_cap = a.sp_cap;
  k.accum = a.accum ? 1u : 0u;
  k.hot_n = a.hot_n;
  k.fold_flag = a.sp_lists ? a.fold_flag : nullptr;
  // row-mask spill entries need every tcpflags group's 8-bin rows aligned in the windows
  k.row_masks = a.spill ? 1u : 0u;
  for (int g = 0; g < a.plan.ngroups; ++g)
    if (a.plan.g[g].family == FAM_TCPFLAGS && !a.plan.g[g].sparse &&
        (a.plan.g[g].nsub != 8 || a.plan.g[g].dense_base < a.spill_lo || (a.plan.g[g].dense_base - a.spill_lo) % 8))
      k.row_masks = 0u;
  k.fold_parity = a.fold_parity;
  k.p = a.plan;
  const bool sketch = a.cms_depth || a.hll_p;
  size_t lds = a.tier1 ? (size_t)a.ipl_bytes + (size_t)a.lds_bins * 4 + kL4ExtraBytes
                       : ((size_t)a.lds_bins + kLdsExtraWords) * 8 + (size_t)k.sp_nwin * 4 +
                             (a.hot_n ? 4 + (size_t)a.hot_n * kHotKeyBytes : 0);
  // the hot-key cache's doorkeeper bitmap takes what LDS is left (2^13 .. 2^18 bits) on the
  // wide-key list path, where any key may otherwise claim an entry
  k.door_log2 = 0;
  if (!a.tier1 && a.hot_n && k.sp_nwin && !a.sparse.compact)
    for (uint32_t l = 18; l >= 13; --l)
      if (lds + ((size_t)1 << (l - 3)) <= kLdsBytes) {
        k.door_log2 = l;
        lds += (size_t)1 << (l - 3);
        break;
      }
  const uint32_t B = a.blocks, T = a.threads;
  hipError_t e;
  // sparse-only plans on the wide-key list path (no dense group, no tcpflags, no sketch,
  // <= 4 groups): wide_kernel
  bool wide = !a.tier1 && !a.dense_ng && !sketch && a.vec && a.hot_n && k.sp_nwin && !a.sparse.compact &&
              a.plan.ngroups >= 1 && a.plan.ngroups <= 4;
  bool excl = true;
  for (int g = 0; wide && g < a.plan.ngroups; ++g) {
    wide = a.plan.g[g].sparse && a.plan.g[g].family != FAM_TCPFLAGS;
    for (int h = 0; h < g; ++h) excl &= a.plan.g[h].family != a.plan.g[g].family;
  }
  if (wide) {
    const bool remote = !a.plan.local, four = a.plan.ngroups > 2;
    // LDS: (remote context) the image of every pod IP when it fits next to a cache of
    // >= kWideIplMinHot entries and a 2^kWideIplMinDoor-bit doorkeeper (the cache halves
    // until it does), counters, cache, then the largest doorkeeper bitmap that fits
    const size_t ctr = (size_t)((k.sp_nwin + 1) / 2) * 8, img = remote && a.ipl ? ((size_t)a.ipl_bytes + 15) & ~15ull : 0;
    int kip = -1;
    if (img) {
      uint32_t hn = k.hot_n;
      while (hn > kWideIplMinHot && img + ctr + (size_t)hn * kHotKeyBytes + ((size_t)1 << (kWideIplMinDoor - 3)) > kLdsBytes)
        hn >>= 1;
      if (img + ctr + (size_t)hn * kHotKeyBytes + ((size_t)1 << (kWideIplMinDoor - 3)) <= kLdsBytes) {
        kip = a.ipl_dense ? 2 : a.ipl_radix ? 1 : 0;
        k.hot_n = hn;
      }
    }
    size_t lw = (kip >= 0 ? img : 0) + ctr + (size_t)k.hot_n * kHotKeyBytes;
    k.door_log2 = 0;
    for (uint32_t l = 18; l >= 13; --l)
      if (lw + ((size_t)1 << (l - 3)) <= kLdsBytes) {
        k.door_log2 = l;
        lw += (size_t)1 << (l - 3);
        break;
      }
    if (kernel) {
      static thread_local char wname[64];
      snprintf(wname, sizeof wname, "wide_kernel<%d, %s, %s, %d>", four ? 4 : 2, remote ? "true" : "false",
               excl ? "true" : "false", kip);
      *kernel = wname;
    }
#define GA_WIDE(NG, R, X, I) e = launch_k(wide_kernel<NG, R, X, I>, k, B, T, lw, st)
#define GA_WIDE_IP(NG, X)                \
  switch (kip) {                          \
    case 2: GA_WIDE(NG, true, X, 2); break; \
    case 1: GA_WIDE(NG, true, X, 1); break; \
    case 0: GA_WIDE(NG, true, X, 0); break; \
    default: GA_WIDE(NG, true, X, -1);     \
  }
    if (four) {
      if (remote) { if (excl) { GA_WIDE_IP(4, true) } else { GA_WIDE_IP(4, false) } }
      else { if (excl) GA_WIDE(4, false, true, -1); else GA_WIDE(4, false, false, -1); }
    } else {
      if (remote) { if (excl) { GA_WIDE_IP(2, true) } else { GA_WIDE_IP(2, false) } }
      else { if (excl) GA_WIDE(2, false, true, -1); else GA_WIDE(2, false, false, -1); }
    }
#undef GA_WIDE_IP
#undef GA_WIDE
    if (e != hipSuccess) return e;
    if (between && (e = hipEventRecord(between, st)) != hipSuccess) return e;
    if (a.defer_folds) {  // lists folded later (launch_folds), or when the device says so
      LaunchArgs r = a;
      r.spill = nullptr;
      r.stage_b = nullptr;
      if (a.stage_defer) r.stage_a = nullptr;
      if (!a.fold_cond) r.sp_lists = nullptr;
      return launch_folds(r, st);
    }
    return launch_folds(a, st);
  }
  int variant = a.tier1 ? 100 + (int)a.dense_ng : (a.dns_compact && a.dense_ng ? 300 : 0) + (int)a.dense_ng;
  if (variant == 304 && a.sig == kSigC5) variant = 305;
  size_t lds_used = lds;
  if (variant == 305 && a.spill && lds + (size_t)a.nwin * (1 + kSpillRing) * 4 <= kLdsBytes) {
    variant = 306;  // spill appends staged in LDS rings
    lds_used = lds + (size_t)a.nwin * (1 + kSpillRing) * 4;
  }
  if (a.tier1) {
    if (a.sig == kSigFwdLdsDropSpill) variant = 200;
    else if (a.sig == kSigFwdLdsDropLds) variant = 201;
    else if (a.sig == kSigFwdLds) variant = 202;
  }
  static const bool trace = getenv("GPUAGG_TRACE") != nullptr;
  if (trace)
    fprintf(stderr, "gpuagg: launch variant=%d tier1=%d sig=0x%x ng=%u L=%u ipl_bytes=%u nwin=%u n=%llu\n",
            variant, (int)a.tier1, a.sig, a.dense_ng, a.lds_bins, a.ipl_bytes, a.nwin,
            (unsigned long long)a.n);
  if (kernel) {
    static thread_local char name[64];
    if (a.tier1)
      snprintf(name, sizeof name, "dense_lds_kernel<%u, %s, %uu, %d>",
               variant >= 200 ? (variant == 202 ? 1u : 2u) : a.dense_ng, a.vec ? "true" : "false",
               variant >= 200 ? a.sig : 0u, a.ipl_dense ? 2 : a.ipl_radix ? 1 : 0);
    else if (a.dense_ng)
      snprintf(name, sizeof name, "dense_local_kernel<%u, %s, %s, %uu%s>", a.dense_ng, a.vec ? "true" : "false",
               a.dns_compact ? "true" : "false", variant >= 305 ? a.sig : 0u, variant == 306 ? ", true" : "");
    else
      snprintf(name, sizeof name, "aggregate_kernel<%s, %s>", a.vec ? "true" : "false", sketch ? "true" : "false");
    *kernel = name;
  }
  switch (variant) {
    case 101: e = launch_lds<1, 0>(a, k, B, T, lds, st); break;
    case 102: e = launch_lds<2, 0>(a, k, B, T, lds, st); break;
    case 104: e = launch_lds<4, 0>(a, k, B, T, lds, st); break;
    case 108: e = launch_lds<8, 0>(a, k, B, T, lds, st); break;
    // compile-time specialised signatures (tier1_signature): the common C2 shapes
    case 200: e = launch_lds<2, kSigFwdLdsDropSpill>(a, k, B, T, lds, st); break;
    case 201: e = launch_lds<2, kSigFwdLdsDropLds>(a, k, B, T, lds, st); break;
    case 202: e = launch_lds<1, kSigFwdLds>(a, k, B, T, lds, st); break;
    case 1: e = a.vec ? launch_k(dense_local_kernel<1, true, false>, k, B, T, lds, st)
                      : launch_k(dense_local_kernel<1, false, false>, k, B, T, lds, st); break;
    case 2: e = a.vec ? launch_k(dense_local_kernel<2, true, false>, k, B, T, lds, st)
                      : launch_k(dense_local_kernel<2, false, false>, k, B, T, lds, st); break;
    case 4: e = a.vec ? launch_k(dense_local_kernel<4, true, false>, k, B, T, lds, st)
                      : launch_k(dense_local_kernel<4, false, false>, k, B, T, lds, st); break;
    case 8: e = a.vec ? launch_k(dense_local_kernel<8, true, false>, k, B, T, lds, st)
                      : launch_k(dense_local_kernel<8, false, false>, k, B, T, lds, st); break;
    // with the compact plan's DNS groups (segment lists)
    case 301: e = a.vec ? launch_k(dense_local_kernel<1, true, true>, k, B, T, lds, st)
                        : launch_k(dense_local_kernel<1, false, true>, k, B, T, lds, st); break;
    case 302: e = a.vec ? launch_k(dense_local_kernel<2, true, true>, k, B, T, lds, st)
                        : launch_k(dense_local_kernel<2, false, true>, k, B, T, lds, st); break;
    case 304: e = a.vec ? launch_k(dense_local_kernel<4, true, true>, k, B, T, lds, st)
                        : launch_k(dense_local_kernel<4, false, true>, k, B, T, lds, st); break;
    case 305: e = a.vec ? launch_k(dense_local_kernel<4, true, true, kSigC5>, k, B, T, lds, st)
                        : launch_k(dense_local_kernel<4, false, true, kSigC5>, k, B, T, lds, st); break;
    case 306: e = a.vec ? launch_k(dense_local_kernel<4, true, true, kSigC5, true>, k, B, T, lds_used, st)
                        : launch_k(dense_local_kernel<4, false, true, kSigC5, true>, k, B, T, lds_used, st); break;
    case 308: e = a.vec ? launch_k(dense_local_kernel<8, true, true>, k, B, T, lds, st)
                        : launch_k(dense_local_kernel<8, false, true>, k, B, T, lds, st); break;
    default:
      if (a.vec)
        e = sketch ? launch_k(aggregate_kernel<true, true>, k, B, T, lds, st)
                   : launch_k(aggregate_kernel<true, false>, k, B, T, lds, st);
      else
        e = sketch ? launch_k(aggregate_kernel<false, true>, k, B, T, lds, st)
                   : launch_k(aggregate_kernel<false, false>, k, B, T, lds, st);
  }
  if (e != hipSuccess) return e;
  if (between && (e = hipEventRecord(between, st)) != hipSuccess) return e;
  if (a.defer_folds) {  // lists folded later (launch_folds), or when the device says so;
    // the tier-1 copies now, unless they accumulate too (stage_defer)
    LaunchArgs r = a;
    r.spill = nullptr;
    r.stage_b = nullptr;
    if (a.stage_defer) r.stage_a = nullptr;
    if (!a.fold_cond) r.sp_lists = nullptr;
    return launch_folds(r, st);
  }
  return launch_folds(a, st);
}

hipError_t launch_folds(const LaunchArgs &a, hipStream_t st, const ForkJoin *fj) {
  hipError_t e;
  const DevDense dd{(unsigned long long *)a.dense_cnt, (unsigned long long *)a.dense_byt};
  // the spill fold + reduce stream: beside the segment fold when both are due
  const bool fork = fj && a.sp_lists && a.sparse.compact && a.spill;
  const hipStream_t sst = fork ? fj->st2 : st;
  if (fork) {
    if ((e = hipEventRecord(fj->fork, st)) != hipSuccess || (e = hipStreamWaitEvent(fj->st2, fj->fork, 0)) != hipSuccess)
      return e;
  }
  // the tier-1 copies are summed by stage_reduce_kernel after the fold (one launch for
  // both reductions); without a fold they get it alone
  const uint32_t ra_x = (a.lds_bins + 255) / 256, ra_y = 8;
  const uint32_t W = 1u << a.win_shift;
  auto reduce = [&](bool with_b) -> hipError_t {
    const uint32_t na = a.stage_a ? ra_x * ra_y : 0u;
    const uint32_t nb = with_b ? (a.nwin * W + 255) / 256 : 0u;
    if (na + nb == 0) return hipSuccess;
    hipLaunchKernelGGL(stage_reduce_kernel, dim3(na + nb), dim3(256), 0, sst, a.stage_a, a.blocks, a.stage_a_stride,
                       a.lds_bins, ra_x, ra_y, a.plan, (const unsigned long long *)a.stage_b, a.nwin,
                       with_b ? a.win_blocks / a.nwin : 0u, W, a.spill_lo, a.dense_len, dd);
    return hipGetLastError();
  };
  if (a.sp_lists && a.sparse.compact) {
    const size_t seg_lds = (size_t)16 << a.sparse.seg_log2;
    if ((e = hipFuncSetAttribute((const void *)sparse_fold_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)seg_lds)) != hipSuccess)
      return e;
    hipLaunchKernelGGL(sparse_fold_kernel, dim3(a.sp_nwin), dim3(1024), seg_lds, st, dev_sparse(a.sparse),
                       (const unsigned long long *)a.sp_lists, a.sp_counts, a.blocks, a.sp_nwin, a.sp_cap);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  } else if (a.sp_lists) {
    const size_t seg_lds = (size_t)8 * kSparseSlotWords << a.sparse.seg_log2;
    if (seg_lds > kLdsBytes) return hipErrorInvalidValue;
    if ((e = hipFuncSetAttribute((const void *)sparse_fold_wide_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)seg_lds)) != hipSuccess)
      return e;
    hipLaunchKernelGGL(sparse_fold_wide_kernel, dim3(a.sp_nwin), dim3(1024), seg_lds, st, dev_sparse(a.sparse),
                       (const unsigned long long *)a.sp_lists, a.sp_counts, a.blocks, a.sp_nwin, a.sp_cap,
                       a.fold_flag, a.fold_parity, a.fold_cond ? a.sp_cap / 2 : 0u);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (!a.spill) return reduce(false);
  e = hipFuncSetAttribute((const void *)spill_window_kernel,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(spill_window_kernel, dim3(a.win_blocks), dim3(1024), (size_t)8 * W, sst,
                     (const uint32_t *)a.spill, a.spill_count, a.blocks, a.spill_cap,
                     a.spill_lo, a.dense_len, W, a.nwin, dd, (unsigned long long *)a.stage_b);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = reduce(a.stage_b != nullptr)) != hipSuccess) return e;
  if (fork) {  // st continues once both folds are done
    if ((e = hipEventRecord(fj->join, sst)) != hipSuccess) return e;
    return hipStreamWaitEvent(st, fj->join, 0);
  }
  return hipSuccess;
}

hipError_t launch_sparse_init(const SparseView &v, size_t slots, hipStream_t st) {
  if (v.compact) return hipMemsetAsync(v.k0, 0, slots * 16, st);
  hipLaunchKernelGGL(sparse_init_kernel, dim3(2048), dim3(256), 0, st,
                     (unsigned long long *)v.k0, slots);
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

hipError_t launch_enrich(const EnrichArgs &a, uint32_t n_cu, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  auto al = [](const void *p) { return ((uintptr_t)p & 15u) == 0; };
  const uint32_t vec = al(a.src) && al(a.dst) && al(a.o_src) && al(a.o_dst);
  const uint64_t lanes = vec ? (a.n + 3) / 4 : a.n;
  const uint64_t need = (lanes + 255) / 256;
  const uint32_t blocks = (uint32_t)(need < (uint64_t)n_cu * 8 ? need : (uint64_t)n_cu * 8);
  hipLaunchKernelGGL(enrich_kernel, dim3(blocks), dim3(256), 0, st,
                     DevIpTable{a.ip_slots, a.ip_mask, a.ip_seed, a.ip_pre, a.ip_blk, 0u, {}}, a.src, a.dst,
                     (uint64_t)a.n, a.o_src, a.o_dst, vec);
  return hipGetLastError();
}

}  // namespace gpuagg
