// Host <-> kernel launch interface (internal).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>
#include <stddef.h>
#include <stdint.h>

#include "gpuagg_internal.h"

namespace gpuagg {

struct ColsView {
  const uint32_t *src_ip, *dst_ip, *bytes, *meta, *ports, *dns_id;
  const uint32_t *tcp_id = nullptr;
  const uint64_t *time_ns = nullptr;
};

struct SparseView {
  uint64_t *k0, *k1, *k2, *cnt, *byt;
  uint32_t mask;
  uint64_t *dropped;
  uint32_t compact;  // 64-bit keys, 2 words (key, count) per slot at k0
  uint32_t seg_log2; // compact: a key probes only its 2^seg_log2-slot segment
  uint32_t narrow;   // wide keys without port / DNS fields: 24-byte list entries
};

struct LaunchArgs {
  ColsView cols;
  size_t n;
  const uint64_t *ip_slots;
  uint32_t ip_mask;
  uint32_t ip_seed;
  const uint16_t *ip_pre;  // radix IP table (null: the bucket table above)
  const uint32_t *ip_blk;
  uint32_t ip_rpn;                       // radix prefixes resolved by compares (0: use ip_pre)
  uint32_t ip_rp[kRadixSmall / 2];
  Plan plan;
  uint64_t *dense_cnt, *dense_byt;
  SparseView sparse;
  uint32_t *cms;
  uint32_t cms_depth, cms_wlog2;
  uint8_t *hll;
  uint32_t hll_p;
  // geometry (see gpuagg_runtime.cpp: plan_launch)
  uint32_t blocks, threads;
  uint64_t chunk;       // records per workgroup, multiple of 4
  bool vec;             // every column 16-byte aligned: dwordx4 loads
  uint32_t lds_bins;    // dense bins [0, lds_bins) privatised in LDS
  uint64_t dense_len;
  uint32_t *spill;      // per-workgroup spill lists (u32 entries), or null
  uint32_t spill_cap;
  uint32_t *spill_count;
  uint32_t win_shift, nwin, win_blocks;  // fold windows of 2^win_shift bins
  uint32_t spill_lo;    // first spilled dense bin (fold windows start here)
  uint32_t dense_ng;    // 0: generic kernel; 1/2/4/8: dense local-context kernel
  bool dns_compact;     // dense kernel also inserts the compact plan's DNS keys (segment lists)
  bool tier1;           // dense kernel with the IP table and u32 bins in LDS
  uint32_t sig;         // tier-1 group signature (kSig*), 0 when the plan has none
  const uint8_t *ipl;
  uint32_t ipl_nb, ipl_seed, ipl_bytes;
  bool ipl_radix;                   // radix image (ipr_build): prefixes below, no nb / seed
  bool ipl_dense;                   // dense radix image (iprd_build): prefixes + descriptors
  uint32_t ipl_npfx, ipl_pfx[kIprMaxPfx], ipl_dr[kIprMaxPfx];
  // staged flushes (null: flush with global atomics)
  uint32_t *stage_a;        // tier-1: [blocks][stage_a_stride] copies of the u32 LDS bins
  uint32_t stage_a_stride;
  uint64_t *stage_b;        // fold: [win_blocks][2^win_shift] window partials
  // compact group-by keys bucketed per table segment (null: inserted in place)
  uint64_t *sp_lists;       // [blocks][sp_nwin][sp_cap] keys
  uint32_t *sp_counts;      // [blocks][sp_nwin]
  uint32_t sp_nwin, sp_cap;
  // deferred folds (gpuagg_runtime.cpp: Pending): accum = the lists hold earlier
  // launches' entries; defer_folds = launch_aggregate leaves the list folds to
  // launch_folds (the tier-1 copies are still summed per launch)
  bool accum;
  bool defer_folds;
  // small deferred launches also keep the tier-1 copies: stage_defer = the copies are
  // summed by the deferred fold (not per launch); stage_accum = this launch's LDS bins
  // start from its workgroup's staged copy (the copies accumulate across launches)
  bool stage_defer;
  bool stage_accum;
  // wide-key lists folded when the device says so: the aggregation kernel records the
  // fullest list in fold_flag[fold_parity] and the per-launch fold skips itself while that
  // is below half the capacity (fold_cond); fold_pending folds unconditionally
  uint32_t *fold_flag;  // [2] u32, zeroed at allocation
  uint32_t fold_parity;
  bool fold_cond;
  uint32_t hot_n;  // aggregate_kernel's LDS hot-key cache entries (0: none)
};
// A second stream for launch_folds: with both compact-key lists and spill lists (C5's
// plan) the spill-window fold and its reduction run on st2 beside the segment fold on st
// (they touch disjoint state), forked after `fork` and joined back through `join`.
struct ForkJoin {
  hipStream_t st2;
  hipEvent_t fork, join;
};
// The list folds of (possibly several deferred) launches with geometry a: the compact
// segment fold, the spill-window fold and its partial reduction.
hipError_t launch_folds(const LaunchArgs &a, hipStream_t st, const ForkJoin *fj = nullptr);

// Raw perf-record decode (gpuagg_decode.hip); kinds match GPUAGG_RAW_* of gpuagg.h.
enum RawKind : int { kRawPacket = 1, kRawDrop = 2 };
struct OutCols {
  uint32_t *src_ip, *dst_ip, *bytes, *meta, *ports, *dns_id;  // ports / dns_id may be null
  uint32_t *tcp_id = nullptr;   // latency columns, may be null
  uint64_t *time_ns = nullptr;
};
struct DecodeArgs {
  int kind;
  const void *raw;         // 16-byte aligned device pointer
  size_t n;                // records
  OutCols out;
  uint64_t *out_of_range;  // device counter: fields that do not fit the meta word
  uint32_t n_cu;
  uint64_t time_offset;    // added to the record times (ktime.MonotonicOffset)
};
hipError_t launch_decode(const DecodeArgs &a, hipStream_t st);

// Standard-mode enriched-flow emission (enrich_kernel, gpuagg_kernels.hip).
struct EnrichArgs {
  const uint64_t *ip_slots;
  uint32_t ip_mask, ip_seed;
  const uint16_t *ip_pre;
  const uint32_t *ip_blk;
  const uint32_t *src, *dst;
  size_t n;
  int32_t *o_src, *o_dst;
};
hipError_t launch_enrich(const EnrichArgs &a, uint32_t n_cu, hipStream_t st);

// Hubble-mode L3/L4 enrichment (gpuagg_hubble.hip).
constexpr uint32_t kIpcEmpty = 0xFFFFFFFFu, kIpcNoMeta = 0xFFFFFFFFu, kIdentityWorld = 2;
enum : uint32_t { kSummaryNone = 0, kSummaryTcp = 1, kSummaryUdp = 2, kSummaryDrop = 3, kSummaryDns = 4 };
struct HubbleArgs {
  const uint4 *table;  // (ip, identity, metadata id, 0); ip kIpcEmpty = free
  uint32_t mask, seed, max_probe;
  const uint32_t *src, *dst, *meta, *dns;
  size_t n;
  uint32_t *o_sid, *o_did, *o_smeta, *o_dmeta, *o_kind, *o_arg;
};
hipError_t launch_hubble(const HubbleArgs &a, uint32_t n_cu, hipStream_t st);

// Node-apiserver latency join (gpuagg_latency.hip).
struct LatEvent {
  uint64_t k0, k1;   // request-oriented key: src | dst << 32, sport | dport << 16 | id << 32
  uint64_t clock;    // record clock (carried entry: its expiry)
  uint64_t seq;      // event number across batches (carried entry: its last touch) -- the
                     // ttlcache's LRU order, needed when the capacity binds
  uint32_t nanos;    // Time.Nanos
  uint32_t bits;     // role 1 request / 2 reply / 3 carried | SYN << 2 | ACK << 3
};
// One live request of the sequential (capacity-bound) pass: the ttlcache item.
struct LatEntry {
  uint64_t k0, k1;
  uint64_t expires;
  uint64_t seq;      // last touch (~0: free)
  uint32_t nanos;
  uint32_t syn;
};
struct LatTouch {  // LRU / expiry queue record (stale once its entry is touched again or freed)
  uint64_t seq;
  uint32_t idx;
  uint32_t pad;
};
constexpr uint64_t kLatLimit = 100000;  // ttlcache.WithCapacity(LIMIT), latency.go:35,120-121
constexpr uint32_t kLatMaxApi = 64;
constexpr uint32_t kLatMaxUnits = 1u << 16;  // front-end units (one wave's contiguous rows each)
constexpr uint64_t kLatTtlNs = 500000000ULL;  // latency.go:34
// state words (u64): clock, pending carried entries, scratch, histograms, no_response
enum : uint32_t {
  kLatClock = 0, kLatPending = 1, kLatCarryOut = 2, kLatClockEnd = 3, kLatEvents = 4,
  kLatSeqBase = 5,     // events numbered so far (LatEvent.seq of this batch's first event)
  kLatHist = 8,        // 11 buckets (le 0, 0.5 .. 4.5, +Inf), count, sum (i64)
  kLatHandshake = 24,  // same layout
  kLatNoResponse = 40,
  kLatCapEvictions = 41,  // requests evicted by the capacity (EvictionReasonCapacityReached)
  kLatCapBatches = 42,    // batches the capacity bound (run by the sequential pass)
  // Words [kLatHist, kLatPeakLive) restart at an epoch reset and are summed by a merge;
  // [kLatPeakLive, kLatStateWords) restart too and are max-merged.
  kLatPeakLive = 43,   // most live requests at any event (the batch's max of the live count)
  kLatStateWords = 48
};
struct LatArgs {
  const uint32_t *src, *dst, *meta, *ports, *tcp_id;
  const uint64_t *time_ns;
  size_t n;
  uint64_t chunk;   // rows per unit (a multiple of 4 when vec)
  uint32_t blocks;  // units (one wave each)
  bool vec;         // meta / tcp_id / time_ns 16-byte aligned: vector loads in the count pass
  const uint32_t *api;
  uint32_t n_api;
  unsigned long long *state;
  uint32_t *blk_cnt;
  unsigned long long *blk_max, *blk_clk;
  uint64_t *blk_base;
  LatEvent *ev;
  unsigned long long *hash_in, *hash_out;
  uint32_t *idx_in, *idx_out;
  const LatEvent *carry_in;
  LatEvent *carry_out;
  // capacity (ttlcache.WithCapacity): live-count check and the sequential pass
  uint64_t limit;
  int32_t *delta, *live;            // [n_events + 1]: +1 / -1 per entry life, its prefix sums
  int32_t *max_live;                // max of live[] (device scalar)
  const uint32_t *carry_order;      // carried entries' positions in LRU (seq) order
};
hipError_t launch_latency_front(const LatArgs &a, hipStream_t st);
hipError_t latency_sort_bytes(size_t n, size_t *bytes);
// The carried entries' LRU order (by last touch): keys / values [2][n] each.
hipError_t latency_carry_order(const LatEvent *carry, size_t n, unsigned long long *keys, uint32_t *vals,
                               void *tmp, size_t tmp_bytes, hipStream_t st);
// The capacity check (sort by key hash, entry lives, live-count scan and its maximum into
// *a.max_live), then -- the host having read that maximum -- the parallel walk's effects
// (limit not reached) or the host's sequential replay (gpuagg_runtime.cpp
// lat_serial_host), then the state update.
hipError_t launch_latency_check(const LatArgs &a, size_t n_events, void *tmp, size_t tmp_bytes,
                                uint32_t enabled, hipStream_t st);
hipError_t launch_latency_walk(const LatArgs &a, size_t n_events, uint32_t enabled, hipStream_t st);
// guard: return at once when the batch's live-count maximum exceeds the limit (a bound
// batch is finished after its host replay, lat_resolve)
hipError_t launch_latency_finish(const LatArgs &a, size_t n_events, bool guard, hipStream_t st);

// Sketch pass (count-min by window partition + HLL), after the metric kernels.
struct SketchArgs {
  ColsView cols;
  size_t n;
  uint64_t chunk;           // records per scatter workgroup
  uint32_t blocks;          // scatter workgroups (= lists per window)
  const uint64_t *ip_slots;
  uint32_t ip_mask, ip_seed;
  const uint16_t *ip_pre;  // radix IP table (null: the bucket table above)
  const uint32_t *ip_blk;
  uint32_t *cms;
  uint32_t cms_depth, cms_wlog2;
  uint32_t win_shift, nwin, cap;  // windows of 2^win_shift columns; nwin 0: direct atomics
  uint16_t *lists;
  uint32_t *counts;
  uint32_t fold_blocks;     // multiple of nwin
  uint8_t *hll;
  uint32_t hll_p;
  uint32_t hll_slots;               // slots covered by the registers
  // HLL two-level bucketing (see SketchK): fine windows of 2^hll_shift pods, super-windows
  // of 2^hll_sshift pods; hll_nsup 0: direct CAS
  uint32_t hll_shift, hll_sshift, hll_nsup, hll_nwin, hll_cap;
  uint32_t *hll_lists, *hll_counts;
  uint32_t hll_b2, hll_cap2;
  uint32_t *hll_lists2, *hll_counts2;
  const uint8_t *ipl;               // LDS image of every pod IP for the source lookup, or null
  uint32_t ipl_nb, ipl_seed, ipl_bytes;
  bool ipl_radix;                   // the image is the radix form (ipl_npfx / ipl_pfx)
  bool ipl_dense;                   // ... the dense radix form (ipl_pfx / ipl_dr)
  uint32_t ipl_npfx, ipl_pfx[kIprMaxPfx], ipl_dr[kIprMaxPfx];
  // which kernels run: the scatter, the folds, or both (kSketchBoth, the default 0); a
  // scatter with accum appends after the fill earlier scatters stored (deferred folds)
  uint32_t passes;
  bool accum;
};
constexpr uint32_t kSketchBoth = 0, kSketchScatter = 1, kSketchFolds = 2;
struct ForkJoin;
// *kernels: the pass's kernels in rocprofv3 spelling joined by "+"; fj (may be null): the
// folds' count-min pass on fj->st2 beside the HLL split + fold on st (disjoint state),
// joined back into st
hipError_t launch_sketch(const SketchArgs &a, hipStream_t st, std::string *kernels, const ForkJoin *fj = nullptr);

// `between` (may be null) is recorded after aggregate_kernel, before the spill fold.
// *kernel (may be null) receives the aggregation kernel's signature as rocprofv3 prints it
// without "void gpuagg::" and the argument list, e.g. "dense_lds_kernel<2, true, 41u>".
hipError_t launch_aggregate(const LaunchArgs &a, hipStream_t st, hipEvent_t between,
                            const char **kernel = nullptr);
hipError_t launch_sparse_init(const SparseView &v, size_t slots, hipStream_t st);
// Clears the dense bins (every endpoint-keyed dense group) and HLL rows (hll may be null)
// of the ndead slots listed at dead (device u32 array).
hipError_t launch_zero_slots(uint64_t *cnt, uint64_t *byt, uint8_t *hll, uint32_t hll_p, const uint32_t *dead,
                             uint32_t ndead, const Plan &p, hipStream_t st);
// Element-wise merge folds: dst += src (u64, u32) and dst = max(dst, src) (u8).
hipError_t launch_merge_add_u64(uint64_t *dst, const uint64_t *src, size_t n, hipStream_t st);
hipError_t launch_merge_add_u32(uint32_t *dst, const uint32_t *src, size_t n, hipStream_t st);
hipError_t launch_merge_max_u8(uint8_t *dst, const uint8_t *src, size_t n, hipStream_t st);
hipError_t launch_sparse_export(const SparseView &v, size_t slots, uint64_t *out, size_t out_cap,
                                uint64_t *counter, hipStream_t st);
hipError_t launch_sparse_import(const SparseView &v, const uint64_t *in, size_t n, hipStream_t st);

// ---- CPU backend (gpuagg_cpu.cpp): the same launches on host memory and threads --------
namespace cpu {
class Engine {
 public:
  explicit Engine(unsigned threads);
  ~Engine();
  // aggregate_kernel's per-record work (dense and group-by updates; no lists, no LDS):
  // into per-thread accumulators, added to the ctx's arrays / table by flush()
  void aggregate(const LaunchArgs &a);
  void flush();
  void drop();  // discards what flush() would add (the state is being reset)
  bool pending() const { return pending_; }
  void sketch(const SketchArgs &s);             // count-min + HLL (relaxed atomics)
  uint64_t decode(const DecodeArgs &a);         // returns the out-of-range rows
  void enrich(const EnrichArgs &a);
  void hubble(const HubbleArgs &a);
  void latency(const LatArgs &a, uint32_t enabled);  // state words in a.state (host)
  void latency_reset();
  unsigned threads() const { return threads_; }

 private:
  struct Part;
  unsigned threads_;
  std::vector<std::unique_ptr<Part>> parts_;
  bool pending_ = false;
  uint64_t dense_len_ = 0;
  uint64_t *dense_cnt_ = nullptr, *dense_byt_ = nullptr;
  SparseView sparse_{};
  std::vector<LatEvent> carry_;  // requests pending across batches
};
void sparse_init(const SparseView &v, size_t slots);
size_t sparse_export(const SparseView &v, size_t slots, uint64_t *out, size_t cap);  // returns entries
void sparse_import(const SparseView &v, const uint64_t *in, size_t n);
void zero_slots(uint64_t *cnt, uint64_t *byt, uint8_t *hll, uint32_t hll_p, const uint32_t *dead, uint32_t ndead,
                const Plan &p);
}  // namespace cpu

}  // namespace gpuagg
