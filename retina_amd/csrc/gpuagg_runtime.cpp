// Host runtime of the flow-aggregation engine: the C ABI of include/gpuagg.h.
//
// Restates, on the host side of the boundary, the parts of the reference that are
// not per-record work:
//  * metric registry resolution  -- Module.updateMetricsContexts (metrics_module.go:205-264)
//    and the constructors / Init of every metric (forward.go:88-118, drops.go:256-286,
//    tcpflags.go:31-51, tcpretrans.go:210-230, dns.go:340-372)
//  * label schemas               -- getLabels (types.go:329-365, forward.go:120-142,
//    drops.go:288-307, tcpflags.go:53-66, tcpretrans.go:232-245, dns.go:374-402)
//  * label values                -- getByDirectionValues (types.go:418-505), enum names
//    (metadata_linux.pb.go:87-95), DNSRcodeToString (flow_utils.go:237-257)
//  * the IP cache snapshot       -- an open-addressed IP -> slot table in HBM
// Per-record work runs in gpuagg_kernels.hip.
#include "../../include/gpuagg.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "gpuagg_build_id.h"
#include "gpuagg_feed.h"
#include "gpuagg_internal.h"
#include "ipl_build.h"
#include "gpuagg_launch.h"

using namespace gpuagg;

namespace {

const char *kDropReasonNames[7] = {"IPTABLE_RULE_DROP", "IPTABLE_NAT_DROP", "TCP_CONNECT_BASIC",
                                   "TCP_ACCEPT_BASIC",  "TCP_CLOSE_BASIC",  "CONNTRACK_ADD_DROP",
                                   "UNKNOWN_DROP"};
const char *kFlagNames[F_COUNT] = {"FIN", "SYNACK", "SYN", "ACK", "RST", "PSH", "URG"};
const char *kRcodeNames[6] = {"NOERROR", "FORMERR", "SERVFAIL", "NXDOMAIN", "NOTIMP", "REFUSED"};
const char *kApiServer = "kubernetes-apiserver";  // pkg/common/types.go:15

std::string drop_reason_name(uint32_t r) { return r < 7 ? kDropReasonNames[r] : std::to_string(r); }
// cilium flow.TrafficDirection names (parity unpinned: cilium proto not in the reference tree)
std::string traffic_direction_name(uint32_t t) {
  switch (t) {
    case 0: return "TRAFFIC_DIRECTION_UNKNOWN";
    case 1: return "INGRESS";
    case 2: return "EGRESS";
  }
  return std::to_string(t);
}
std::string ip_string(uint32_t ip) {  // utils.Int2ip + net.IP.String()
  char b[20];
  snprintf(b, sizeof b, "%u.%u.%u.%u", ip & 255u, (ip >> 8) & 255u, (ip >> 16) & 255u, ip >> 24);
  return b;
}

std::string lower(const char *s) {
  std::string o(s ? s : "");
  for (auto &c : o) c = (char)tolower((unsigned char)c);
  return o;
}

struct SlotAttr {
  std::string ns, pod, wk_kind, wk_name;
  bool has_owner = false;
  bool api = false;
  bool in_use = true;  // false once retired (gpuagg_retire_slots); the id is then reusable
};

struct DnsAttr {
  uint32_t rcode, nresp;
  std::string qtypes, query, ips;
  bool in_use = true;  // false once retired (gpuagg_dns_retire); the id is then reusable
  bool idle = false;   // no key referenced it at the last gpuagg_dns_retire (retired at the next)
};

enum ValueKind { VK_COUNT, VK_BYTES };

// One registered metric object (the value type of Module.registry).
struct Instance {
  std::string registry_name;  // MetricsContextOptions.MetricName
  uint8_t family;
  ValueKind vk;
  std::string vec_name;  // "networkobservability_adv_..."
  std::vector<std::string> label_names;
  bool active;      // emits series (Init created a vector and update() matches)
  bool adv_enable;  // forward remote: ctx values only when advanced
  bool has_src, has_dst;
  uint8_t src_opts, dst_opts;
  int group;
};

struct Group {
  uint8_t family, src_opts, dst_opts;
  bool sparse;
  uint32_t nsub, key_mode;
  uint64_t dense_base, nkeys;
};

// One Prometheus series of a snapshot: its family (the registered metric object), its
// label values (NUL-terminated, in the family's label order, in one of the result's
// arenas) and its value.
struct SeriesRec {
  uint32_t fam;
  uint32_t arena;
  uint64_t off;
  uint64_t value;
  uint64_t tok;  // its label values' sort tokens (render_series), in the same arena's token list
  uint32_t len;  // bytes of its label values in the arena (NULs included)
  uint32_t esc;  // a value holds a byte the exposition escapes (\\ " newline)
};

// One canonical id's labels at render time: its values' sort tokens and where its
// pre-rendered values lie (one cache line per id for render_series' random lookups).
struct LabelRec {
  uint32_t tok[5];
  uint32_t len;
  uint64_t off;
};

// Canonical ids of the slot attributes a side's options render (namespace / pod /
// workload; the service label is constant): id[slot1] (slot1 0 or past the table:
// "unknown") and a representative slot1 per id; rebuilt when the slots change.
struct SlotCanon {
  std::vector<uint32_t> id, rep;
  // per id: rank of its namespace / podname / workload kind / workload name string among
  // the ids' (exposition sort tokens)
  // rendered values (ctx_values_into of the mask, NUL-terminated) at blk[rec[id].off], tokens
  // of namespace / podname / workload kind / workload name in rec[id].tok
  std::vector<char> blk;
  std::vector<LabelRec> rec;
  uint64_t version = ~0ull;
};

struct ResultFamily {
  std::string metric;
  std::vector<std::string> names;
  std::vector<const char *> name_ptrs;
  std::vector<uint32_t> by_name;  // label positions in name order (client_golang sorts pairs)
  const char *type = "", *help = "";
};

// A metric family's Prometheus type and Help text, as the reference's Init creates its
// vector (forward.go:18-26,47-64; drops.go:18-23,42-60; tcpflags.go:18-24,43-51;
// tcpretrans.go:18-24,43-51: GaugeVec; dns.go:21-30,50-66: CounterVec).
struct FamilyInfo {
  const char *type, *help;
};
FamilyInfo family_info(const std::string &vec) {
  if (vec == "adv_forward_count") return {"gauge", "Total number of forwarded packets"};
  if (vec == "adv_forward_bytes") return {"gauge", "Total number of forwarded bytes"};
  if (vec == "adv_drop_count") return {"gauge", "Total number of dropped packets"};
  if (vec == "adv_drop_bytes") return {"gauge", "Total number of dropped bytes"};
  if (vec == "adv_tcpflags_count") return {"gauge", "Total number of packets by TCP flag"};
  if (vec == "adv_tcpretrans_count") return {"gauge", "Total number of TCP retransmitted packets"};
  if (vec == "adv_dns_request_count") return {"counter", "Total number of DNS query packets"};
  if (vec == "adv_dns_response_count") return {"counter", "Total number of DNS response packets"};
  return {"untyped", ""};
}

// Options of one MetricsContextOptions as last applied (the reconcile no-op comparison).
struct OptCopy {
  std::string name;
  std::vector<std::string> src, dst;
};

struct LKey {
  uint32_t w[8];  // view, prefix (direction / reason / flag / DNS payload), src ip / attrs / port, dst ...
  bool operator==(const LKey &o) const { return memcmp(w, o.w, sizeof w) == 0; }
};
struct LKeyHash {
  size_t operator()(const LKey &k) const {
    uint64_t h = 0x8BADF00DULL;
    for (int i = 0; i < 8; i += 2) h = fmix64(h ^ ((uint64_t)k.w[i] | ((uint64_t)k.w[i + 1] << 32)));
    return (size_t)h;
  }
};
struct LItem {
  LKey k;
  uint64_t cnt, byt;
};

// std::allocator whose resize leaves new elements default-initialized (no zero fill:
// every element is written right after)
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U> &) {}
  template <class U>
  void construct(U *p) noexcept {
    ::new ((void *)p) U;
  }
  template <class U, class... A>
  void construct(U *p, A &&...a) {
    ::new ((void *)p) U(std::forward<A>(a)...);
  }
};
using SeriesVec = std::vector<SeriesRec, NoInitAlloc<SeriesRec>>;

// The scrape's large buffers, kept mapped between snapshots: a result borrows them and
// gpuagg_result_free hands them back, so the next scrape writes into pages that are
// already faulted in (c4-remote's scrape touches ~3 GB per snapshot; on the GPU box the
// page faults of fresh buffers were most of its host time).  Shared by the ctx and its
// results, so a result may outlive its ctx.
struct ScrapePool {
  std::mutex mu;
  std::vector<std::vector<char>> arenas;
  std::vector<std::vector<uint32_t>> toks;
  SeriesVec series;
  std::unique_ptr<char[]> text;
  size_t text_cap = 0;
};

}  // namespace

struct gpuagg_result {
  std::vector<ResultFamily> fam;  // one per registered metric object
  SeriesVec series;
  std::vector<std::vector<char>> arenas;
  std::vector<std::vector<uint32_t>> toks;  // per arena: label sort tokens (render_series)
  std::shared_ptr<ScrapePool> pool;         // where the buffers go back
  // series i's label values: value_ptrs[voff[i] ...], built on the first gpuagg_result_series
  // (the exposition text walks the arenas itself)
  mutable std::vector<const char *> value_ptrs;
  mutable std::vector<uint64_t> voff;
  mutable std::once_flag ptrs_once;
  uint64_t dropped = 0;
  // families rendered outside `series` (the latency histograms / no_response counter):
  // name -> exposition text block
  std::map<std::string, std::string> extra_text;
  // gpuagg_result_render_text's output, rendered once (callers size, then fill)
  mutable std::unique_ptr<char[]> text;  // text_len bytes + NUL, text_cap allocated
  mutable size_t text_len = 0, text_cap = 0;
  mutable std::once_flag text_once;  // render_text runs once, whichever reader comes first
};

struct gpuagg_ctx {
  gpuagg_config cfg{};
  int device = 0;
  // CPU backend (GPUAGG_FLAG_CPU_BACKEND, gpuagg_cpu.cpp): every "device" buffer below is
  // host memory and the launches run on host threads; no HIP call is made
  std::unique_ptr<gpuagg::cpu::Engine> cpu;
  bool host_timing = false;  // CPU backend: gpuagg_set_timing measures the host launches
  // in-process RCCL communicators of the last gpuagg_merge this ctx was the target of
  // (one per device of the merge, created once per device list)
  std::vector<int> rccl_devs;
  std::vector<ncclComm_t> rccl_comms;
  hipStream_t stream = nullptr;
  std::string err;

  // registry / plan
  bool remote = false;
  std::vector<Instance> inst;
  std::vector<Group> groups;
  Plan plan{};

  // identity dictionaries
  std::map<std::tuple<std::string, std::string, std::string, std::string, int>, int32_t> slot_ids;
  std::vector<SlotAttr> slots;
  std::vector<int32_t> free_slots;  // retired ids, reused first by gpuagg_slot_intern
  uint32_t key_cap = 0;             // slots covered by the dense counters and HLL rows
  std::vector<std::pair<uint32_t, int32_t>> installed;  // the installed IP -> slot map
  std::vector<OptCopy> cur_opts;    // options of the last applied reconcile
  bool have_opts = false;
  // native IP cache (cache.go): endpoints "ns/name" -> (slot, IPs); services, nodes -> IP
  struct CacheEp {
    int32_t slot;
    std::vector<uint32_t> ips;
  };
  std::unordered_map<std::string, CacheEp> ep_map;
  std::unordered_map<uint32_t, std::string> ip_to_ep;
  std::unordered_map<std::string, uint32_t> svc_map, node_map;
  std::unordered_map<uint32_t, std::string> ip_to_svc, ip_to_node;
  std::unordered_map<std::string, uint32_t> dns_ids;
  std::vector<DnsAttr> dns;
  std::vector<uint32_t> free_dns;  // retired DNS ids, reused (lowest first) by gpuagg_dns_intern
  // label-canonical DNS payloads, kept at intern time: request series render (qtypes,
  // query), response series (rcode name, qtypes, query, ips, answers)
  std::unordered_map<std::string, uint32_t> dns_req_canon, dns_resp_canon;
  std::vector<uint32_t> dns_req_id, dns_resp_id, dns_req_rep, dns_resp_rep;
  // per canonical payload: sort tokens of request (qtypes, query) / response (rcode, qtypes,
  // query, ips, answers) labels and its block below; rebuilt when the table has grown
  std::vector<LabelRec> dns_req_rec, dns_resp_rec;
  // the canonical payloads' label values, rendered at intern time (NUL-terminated, in
  // label order): block of id i = [*_boff[i], *_boff[i + 1])
  std::vector<char> dns_req_blk, dns_resp_blk;
  std::vector<uint64_t> dns_req_boff{0}, dns_resp_boff{0};
  // canonical slot attributes per option mask (snapshot), valid for slots_version
  std::map<uint8_t, SlotCanon> slot_canon;
  // the scrape's buffers, reused between snapshots (results borrow the large ones)
  std::shared_ptr<ScrapePool> scrape_pool = std::make_shared<ScrapePool>();
  struct AggScratch {
    std::vector<std::vector<std::vector<LItem>>> parts;
    std::vector<std::vector<LItem>> tab;
    std::vector<SeriesVec> out;
  } agg_scratch;
  uint64_t slots_version = 0;

  // IP table
  uint64_t *d_ip = nullptr;
  // radix IP table (few /16 prefixes): prefix -> block, blocks of 64k u32 entries
  uint16_t *d_rpre = nullptr;
  uint32_t *d_rblk = nullptr;
  size_t rblk_alloc = 0;
  bool radix = false;
  uint32_t radix_n = 0;                   // prefixes (blocks) of the radix table
  uint32_t radix_pfx[kRadixSmall / 2] = {};  // their values when radix_n <= kRadixSmall
  size_t ip_cap = 0;  // slots
  uint32_t ip_seed = 0;
  // LDS image of the IP table for the tier-1 dense kernel (empty: not available)
  uint8_t *d_ipl = nullptr;
  size_t ipl_alloc = 0;
  // Hubble ipcache image (gpuagg_hubble.hip)
  uint4 *d_ipc = nullptr;
  size_t ipc_cap = 0;
  uint32_t ipc_seed = 0, ipc_max_probe = 0;
  // node-apiserver latency join (gpuagg_latency.hip)
  uint32_t lat_enabled = 0;  // bit 0 latency, 1 handshake, 2 no_response
  std::vector<uint32_t> api_ips;
  uint32_t *d_api = nullptr;
  unsigned long long *d_lat = nullptr;  // kLatStateWords
  uint32_t *d_lat_blk_cnt = nullptr;
  unsigned long long *d_lat_blk_max = nullptr, *d_lat_blk_clk = nullptr;
  uint64_t *d_lat_blk_base = nullptr;
  size_t lat_blk_alloc = 0;
  LatEvent *d_lat_ev = nullptr;
  size_t lat_ev_alloc = 0;
  unsigned long long *d_lat_hash = nullptr;  // [2][lat_ev_alloc]: sort in, sort out
  uint32_t *d_lat_idx = nullptr;
  LatEvent *d_lat_carry[2] = {nullptr, nullptr};
  size_t lat_carry_alloc = 0;
  int lat_carry_cur = 0;
  uint64_t lat_carry_bound = 0;  // >= entries currently carried
  void *d_lat_tmp = nullptr;
  size_t lat_tmp_alloc = 0;
  // capacity (ttlcache LIMIT): live-count check buffers and the sequential pass's ttlcache
  int32_t *d_lat_delta = nullptr;   // [2][lat_ev_alloc + 1]: entry lives, live counts
  int32_t *d_lat_max_live = nullptr;
  unsigned long long *d_lat_okeys = nullptr;  // carried entries' LRU sort: [2][lat_carry_alloc]
  uint32_t *d_lat_ovals = nullptr;
  size_t lat_order_alloc = 0;
  uint64_t *h_lat_n = nullptr;   // pinned: state words [kLatPending, kLatEvents] of the batch
                                 // and, at [kLatReadWords], the batch's live-count maximum
  // the last batch's capacity decision, read at the next synchronisation (lat_resolve)
  struct LatPend {
    bool active = false;
    LatArgs a{};
    uint64_t ne = 0, pend = 0;
  } lat_pend;
  uint64_t lat_peak_pending = 0; // most requests carried into a batch since the reconcile
  int64_t time_offset = 0;       // ktime.MonotonicOffset added to decoded record times
  uint8_t *d_ipl_all = nullptr;  // every pod IP incl. the apiserver (sketch pass)
  size_t ipl_all_alloc = 0;
  uint32_t ipl_all_nb = 0, ipl_all_seed = 0, ipl_all_bytes = 0;
  bool ipl_all_radix = false, ipl_all_dense = false;  // image form (build_lds_image)
  uint32_t ipl_all_npfx = 0, ipl_all_pfx[kIprMaxPfx] = {}, ipl_all_dr[kIprMaxPfx] = {};
  uint32_t ipl_nb = 0, ipl_seed = 0, ipl_bytes = 0;
  // the tier-1 image: dense radix, radix or cuckoo form (build_lds_image)
  bool ipl_radix = false, ipl_dense = false;
  uint32_t ipl_npfx = 0, ipl_pfx[kIprMaxPfx] = {}, ipl_dr[kIprMaxPfx] = {};
  uint64_t ip_version = 0;

  // dense counters
  uint64_t *d_dense_cnt = nullptr, *d_dense_byt = nullptr;
  size_t dense_len = 0;

  // sparse table
  SparseView sv{};
  size_t sparse_slots = 0;
  uint64_t *d_counter = nullptr;  // export counter
  uint64_t *d_export = nullptr;
  size_t export_cap = 0;

  // sketches
  uint32_t *d_cms = nullptr;
  size_t cms_len = 0;
  uint8_t *d_hll = nullptr;
  size_t hll_len = 0;
  std::vector<uint32_t> h_cms;
  std::vector<uint8_t> h_hll;

  // Device staging for host-fed batches, double-buffered: batch k+1's H2D copy (on
  // copy_stream) overlaps batch k's aggregation (on stream).  `copied` is recorded on
  // copy_stream after the copy, `released` on stream after the last kernel reading it.
  struct Staging {
    uint32_t *cols[6] = {};
    uint32_t *tcp_id = nullptr;  // latency columns
    uint64_t *time_ns = nullptr;
    uint8_t *raw = nullptr;
    size_t raw_alloc = 0;
    hipEvent_t copied = nullptr, released = nullptr;
    bool in_use = false;
  } stg[2];
  size_t staging_cap = 0;
  int next_stg = 0;
  hipStream_t copy_stream = nullptr;
  // deferred folds: the spill-window fold beside the segment fold (launch_folds' ForkJoin)
  hipStream_t fold_stream = nullptr;
  hipEvent_t fold_fork = nullptr, fold_join = nullptr;
  std::vector<gpuagg_batch *> batches;
  std::string kernel_name;  // aggregation kernel of the last launch (rocprofv3 spelling)
  std::string sketch_kernel_name;  // kernels of the last sketch pass, joined by "+"

  // stats / timing
  gpuagg_stats stats{};
  bool timing = false;
  std::vector<std::array<hipEvent_t, 3>> pending_events;  // start, after aggregate, after fold
  // Timing events cost ~4 us of idle GPU each (a barrier packet): consecutive launches share
  // one -- a launch's start is the previous launch's end event when nothing else was
  // enqueued on the stream in between (tm_chain; ENQ() clears it at every other enqueue).
  hipEvent_t tm_end = nullptr;
  bool tm_chain = false;
  uint32_t n_cu = 256;
  // dense spill lists (per workgroup) for bins beyond the LDS window
  uint32_t *d_spill = nullptr;
  size_t spill_alloc = 0;
  uint32_t *d_spill_count = nullptr;
  size_t spill_count_alloc = 0;
  // staged flushes: per-workgroup LDS bins (tier-1) and per-partition fold windows
  uint32_t *d_stage_a = nullptr;
  size_t stage_a_alloc = 0;
  uint32_t *d_fold_flag = nullptr;  // device-conditional wide-list folds: [2] fullest list
  uint32_t fold_parity = 0;
  // Deferred list folds: the spill / segment lists of consecutive launches with one
  // geometry accumulate and are folded once (fold_pending) -- per scrape epoch rather
  // than per batch, so C5's fixed 128 MiB table pass is paid once per sync.
  struct Pending {
    bool active = false;
    LaunchArgs a{};         // geometry and lists of the launches waiting for their fold
    uint64_t budget = 0;    // records per workgroup the lists were sized for
    uint64_t rpb = 0;       // records per workgroup appended so far
  } pend;
  // Deferred sketch folds: small launches' count-min / HLL scatter lists accumulate (the
  // scatter starts from the stored fill) and cms_fold / hll_split / hll_fold run once.
  struct SketchPending {
    bool active = false;
    SketchArgs s{};       // geometry and lists of the waiting scatters
    uint64_t budget = 0;  // records per scatter workgroup the lists were sized for
    uint64_t rpb = 0;     // records per workgroup appended so far
  } sk_pend;
  bool defer_folds = true;
  uint64_t wide_list_bytes = 0;  // wide-key list budget (gpuagg_create)
  std::vector<std::array<hipEvent_t, 2>> pending_fold;  // deferred fold start, end
  int32_t *d_enrich = nullptr;  // gpuagg_submit_enrich: [2][cap] endpoint slots
  size_t enrich_alloc = 0;
  hipEvent_t enrich_done = nullptr;
  uint64_t *d_stage_b = nullptr;
  size_t stage_b_alloc = 0;
  // raw perf-record decode (gpuagg_decode.hip)
  uint64_t *d_decode_oor = nullptr;  // out-of-range field counter
  std::vector<std::array<hipEvent_t, 2>> pending_decode;  // decode start, end
  // sketch pass (count-min window lists)
  uint16_t *d_sk_lists = nullptr;
  size_t sk_lists_alloc = 0;
  uint32_t *d_sk_counts = nullptr;
  size_t sk_counts_alloc = 0;
  uint64_t *d_sp_lists = nullptr;
  size_t sp_lists_alloc = 0;
  uint32_t *d_sp_counts = nullptr;
  size_t sp_counts_alloc = 0;
  uint32_t *d_hll_lists = nullptr;
  size_t hll_lists_alloc = 0;
  uint32_t *d_hll_counts = nullptr;
  size_t hll_counts_alloc = 0;
  uint32_t *d_hll_lists2 = nullptr;
  size_t hll_lists2_alloc = 0;
  uint32_t *d_hll_counts2 = nullptr;
  size_t hll_counts2_alloc = 0;
  std::vector<std::array<hipEvent_t, 2>> pending_sketch;  // sketch scatter launch start, end
  uint64_t pending_sketch_submits = 0;  // submits those launches belong to (sketch_launches)
  // node-wide feeds over this context (gpuagg_feed.cpp): detached by gpuagg_destroy
  std::vector<gpuagg_raw_feed *> feeds;
  uint64_t host_decode_oor = 0;  // out-of-range rows the feeds decoded on the host
  uint64_t *h_sync_words = nullptr;  // pinned: gpuagg_sync's counter readback [decode oor, sparse dropped]
};

// ------------------------------------------------------------------------------------
namespace {

int fail(gpuagg_ctx *c, int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(c, expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      return fail((c), GPUAGG_EDEVICE, "%s failed: %s", #expr, hipGetErrorString(_e));   \
  } while (0)

// Marks the stream as used by something other than launch()'s timed kernels.
#define ENQ(c) ((c)->tm_chain = false)

int bind(gpuagg_ctx *c) {
  if (c->cpu) return GPUAGG_OK;
  HIPCHK(c, hipSetDevice(c->device));
  return GPUAGG_OK;
}

// ---- execution layer: the ctx's gfx950 device, or (CPU backend) host memory ------------
hipError_t x_sync(gpuagg_ctx *c, hipStream_t st) { return c->cpu ? hipSuccess : hipStreamSynchronize(st); }
hipError_t x_copy(gpuagg_ctx *c, void *dst, const void *src, size_t n, hipMemcpyKind k) {
  if (!c->cpu) return hipMemcpy(dst, src, n, k);
  if (n) memmove(dst, src, n);
  return hipSuccess;
}
hipError_t x_copy_async(gpuagg_ctx *c, void *dst, const void *src, size_t n, hipMemcpyKind k, hipStream_t st) {
  ENQ(c);
  if (!c->cpu) return hipMemcpyAsync(dst, src, n, k, st);
  if (n) memmove(dst, src, n);
  return hipSuccess;
}
hipError_t x_set_async(gpuagg_ctx *c, void *p, int v, size_t n, hipStream_t st) {
  ENQ(c);
  if (!c->cpu) return hipMemsetAsync(p, v, n, st);
  if (n) memset(p, v, n);
  return hipSuccess;
}
// pinned host memory (device mode) / plain host memory (CPU backend)
hipError_t x_host_alloc(gpuagg_ctx *c, void **p, size_t n) {
  if (!c->cpu) return hipHostMalloc(p, n, hipHostMallocDefault);
  *p = calloc(1, n ? n : 1);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
void x_host_free(gpuagg_ctx *c, void *p) {
  if (!p) return;
  if (c->cpu) free(p);
  else hipHostFree(p);
}

template <class T>
int dev_alloc(gpuagg_ctx *c, T **p, size_t count) {
  *p = nullptr;
  if (!count) return GPUAGG_OK;
  if (c->cpu) {  // 64-byte aligned like device allocations (vector loads, 16-byte slots)
    const size_t bytes = (count * sizeof(T) + 63) & ~(size_t)63;
    void *q = aligned_alloc(64, bytes);
    if (!q) return fail(c, GPUAGG_ENOMEM, "aligned_alloc(%zu bytes)", bytes);
    memset(q, 0, bytes);
    *p = (T *)q;
    return GPUAGG_OK;
  }
  hipError_t e = hipMalloc((void **)p, count * sizeof(T));
  if (e != hipSuccess)
    return fail(c, GPUAGG_ENOMEM, "hipMalloc(%zu bytes): %s", count * sizeof(T), hipGetErrorString(e));
  return GPUAGG_OK;
}

template <class T>
void dev_free(gpuagg_ctx *c, T *&p) {
  if (p) {
    if (c->cpu) free((void *)p);
    else hipFree((void *)p);
  }
  p = nullptr;
}

// Grows a lazily allocated device buffer to at least `count` elements.
template <class T>
int ensure_buf(gpuagg_ctx *c, T **p, size_t *alloc, size_t count) {
  if (count <= *alloc) return GPUAGG_OK;
  if (*p) x_sync(c, c->stream);  // in-flight launches may still use the old buffer
  dev_free(c, *p);
  *alloc = 0;
  if (int rc = dev_alloc(c, p, count)) return rc;
  *alloc = count;
  return GPUAGG_OK;
}

uint8_t parse_opts(const char *const *labels, uint32_t n) {  // NewCtxOption (types.go:300-327)
  uint8_t o = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const std::string s = lower(labels[i]);
    if (s == "ip") o |= OPT_IP;
    else if (s == "namespace") o |= OPT_NS;
    else if (s == "podname") o |= OPT_POD;
    else if (s == "workload") o |= OPT_WL;
    else if (s == "service") o |= OPT_SVC;
    else if (s == "port") o |= OPT_PORT;
  }
  return o;
}

void ctx_label_names(uint8_t opts, const char *prefix, std::vector<std::string> &out) {
  std::string p(prefix);
  if (opts & OPT_IP) out.push_back(p + "ip");
  if (opts & OPT_NS) out.push_back(p + "namespace");
  if (opts & OPT_POD) out.push_back(p + "podname");
  if (opts & OPT_WL) {
    out.push_back(p + "workload_kind");
    out.push_back(p + "workload_name");
  }
  if (opts & OPT_SVC) out.push_back(p + "service");
  if (opts & OPT_PORT) out.push_back(p + "port");
}

// getByDirectionValues for one side tuple (types.go:418-505).
void ctx_values(const gpuagg_ctx *c, uint8_t opts, uint32_t ip, uint32_t slot1, uint32_t port17,
                std::vector<std::string> &out) {
  const SlotAttr *a = (slot1 && slot1 - 1 < c->slots.size()) ? &c->slots[slot1 - 1] : nullptr;
  if (opts & OPT_IP) out.push_back(ip_string(ip));
  if (opts & OPT_NS) out.push_back(a ? a->ns : "unknown");
  if (opts & OPT_POD) out.push_back(a ? a->pod : "unknown");
  if (opts & OPT_WL) {
    if (a && a->has_owner) {
      out.push_back(a->wk_kind);
      out.push_back(a->wk_name);
    } else {
      out.push_back("unknown");
      out.push_back("unknown");
    }
  }
  if (opts & OPT_SVC) out.push_back("unknown");
  if (opts & OPT_PORT) out.push_back((port17 & 0x10000u) ? std::to_string(port17 & 0xFFFFu) : "unknown");
}

void free_batch_cols(gpuagg_ctx *c, gpuagg_batch *b) {
  for (uint32_t **p : {&b->cols.src_ip, &b->cols.dst_ip, &b->cols.bytes, &b->cols.meta,
                       &b->cols.ports, &b->cols.dns_id, &b->cols.tcp_id}) {
    x_host_free(c, *p);
    *p = nullptr;
  }
  x_host_free(c, b->cols.time_ns);
  b->cols.time_ns = nullptr;
}

int ensure_staging(gpuagg_ctx *c, size_t cap) {
  if (cap <= c->staging_cap) return GPUAGG_OK;
  if (c->staging_cap) {  // in-flight copies / launches may use the old columns
    HIPCHK(c, x_sync(c, c->copy_stream));
    HIPCHK(c, x_sync(c, c->stream));
  }
  c->staging_cap = 0;
  for (auto &s : c->stg) {
    for (auto &p : s.cols) dev_free(c, p);
    dev_free(c, s.tcp_id);
    dev_free(c, s.time_ns);
    for (auto &p : s.cols)
      if (int rc = dev_alloc(c, &p, cap)) return rc;
    if (int rc = dev_alloc(c, &s.tcp_id, cap)) return rc;
    if (int rc = dev_alloc(c, &s.time_ns, cap)) return rc;
  }
  c->staging_cap = cap;
  return GPUAGG_OK;
}

// The next staging buffer, once the kernels that read it last have finished.
int acquire_staging(gpuagg_ctx *c, gpuagg_ctx::Staging **out) {
  gpuagg_ctx::Staging &s = c->stg[c->next_stg];
  c->next_stg ^= 1;
  if (s.in_use) HIPCHK(c, hipEventSynchronize(s.released));
  s.in_use = false;
  *out = &s;
  return GPUAGG_OK;
}

// After the H2D copies into s were enqueued on copy_stream: the aggregation stream waits
// for them, `launch_fn` enqueues the kernels, s is released behind them, and the call
// returns once the copies (not the kernels) are complete, so the caller's host buffer
// may be refilled while the aggregation runs.
// With `host_done` (the feeds' async submits) that event is recorded behind the copies and
// the call returns without waiting for them.
template <class F>
int run_staged(gpuagg_ctx *c, gpuagg_ctx::Staging &s, F &&launch_fn, hipEvent_t host_done = nullptr) {
  HIPCHK(c, hipEventRecord(s.copied, c->copy_stream));
  if (host_done) HIPCHK(c, hipEventRecord(host_done, c->copy_stream));
  HIPCHK(c, hipStreamWaitEvent(c->stream, s.copied, 0));
  int rc = launch_fn();
  HIPCHK(c, hipEventRecord(s.released, c->stream));
  s.in_use = true;
  if (host_done) {
    c->stats.async_returns += 1;
    return rc;
  }
  HIPCHK(c, hipEventSynchronize(s.copied));
  if (hipEventQuery(s.released) == hipErrorNotReady) c->stats.async_returns += 1;
  return rc;
}

// Timing-only events: recording one with the default system-scope fence writes back and
// invalidates the caches between kernels (measured ~5.5 us of idle GPU per event at C2,
// profiles/round2/r4a_*); results are published by gpuagg_sync's stream sync, not by
// these events.
constexpr unsigned kTimingEventFlags = hipEventDisableSystemFence;

// Folds the lists of the deferred launches (no-op when none are waiting).  Every reader
// of the counters or the group-by table calls it first: gpuagg_sync (and through it the
// snapshot), state export, merge, slot retirement and dense re-layout.
int fold_pending_sketch(gpuagg_ctx *c);

// The ctx's second stream for folds that run side by side (launch_folds, launch_sketch).
int fold_fork_join(gpuagg_ctx *c, ForkJoin *fj) {
  if (!c->fold_stream) {
    HIPCHK(c, hipStreamCreateWithFlags(&c->fold_stream, hipStreamNonBlocking));
    HIPCHK(c, hipEventCreateWithFlags(&c->fold_fork, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->fold_join, hipEventDisableTiming));
  }
  *fj = ForkJoin{c->fold_stream, c->fold_fork, c->fold_join};
  return GPUAGG_OK;
}

// The aggregation launches' deferred lists only (their own budget ran out: the sketch
// lists keep theirs).
int fold_pending_dense(gpuagg_ctx *c) {
  if (c->cpu || !c->pend.active) return GPUAGG_OK;
  c->pend.active = false;
  LaunchArgs f = c->pend.a;
  if (!f.stage_defer) f.stage_a = nullptr;  // summed per launch, unless the copies accumulate
  f.stage_accum = false;
  f.defer_folds = false;
  f.fold_cond = false;  // unconditional (the flags are left to the launches)
  std::array<hipEvent_t, 2> ev{};
  if (c->timing) {
    for (auto &e : ev) HIPCHK(c, hipEventCreateWithFlags(&e, kTimingEventFlags));
    HIPCHK(c, hipEventRecord(ev[0], c->stream));
  }
  ENQ(c);
  ForkJoin fj{};
  const bool fork = f.sp_lists && f.sparse.compact && f.spill;
  if (fork)
    if (int rc = fold_fork_join(c, &fj)) return rc;
  HIPCHK(c, launch_folds(f, c->stream, fork ? &fj : nullptr));
  if (c->timing) {
    HIPCHK(c, hipEventRecord(ev[1], c->stream));
    c->pending_fold.push_back(ev);
  }
  return GPUAGG_OK;
}

int lat_resolve(gpuagg_ctx *c);

int fold_pending(gpuagg_ctx *c) {
  if (c->cpu) {  // the host threads' accumulators into the ctx's counters and table
    c->cpu->flush();
    return GPUAGG_OK;
  }
  if (int rc = lat_resolve(c)) return rc;
  if (int rc = fold_pending_sketch(c)) return rc;
  return fold_pending_dense(c);
}

// The state is being cleared: the waiting lists are discarded with it.
void drop_pending(gpuagg_ctx *c) {
  c->pend.active = false;
  c->sk_pend.active = false;
  if (c->cpu) c->cpu->drop();
}

int reset_state(gpuagg_ctx *c) {
  drop_pending(c);
  if (c->dense_len) {
    HIPCHK(c, x_set_async(c, c->d_dense_cnt, 0, c->dense_len * 8, c->stream));
    HIPCHK(c, x_set_async(c, c->d_dense_byt, 0, c->dense_len * 8, c->stream));
  }
  if (c->sparse_slots) {
    HIPCHK(c, x_set_async(c, c->sv.dropped, 0, 8, c->stream));
    if (c->cpu) cpu::sparse_init(c->sv, c->sparse_slots);
    else {
      ENQ(c);
      HIPCHK(c, launch_sparse_init(c->sv, c->sparse_slots, c->stream));
    }
  }
  if (c->cms_len) HIPCHK(c, x_set_async(c, c->d_cms, 0, c->cms_len * 4, c->stream));
  if (c->hll_len) HIPCHK(c, x_set_async(c, c->d_hll, 0, c->hll_len, c->stream));
  HIPCHK(c, x_sync(c, c->stream));
  return GPUAGG_OK;
}

int ensure_sparse(gpuagg_ctx *c) {
  if (c->sparse_slots) return GPUAGG_OK;
  // (the compact layout needs 2 of the 8 words per slot; one allocation serves both)
  const uint32_t lg = c->cfg.sparse_capacity_log2 ? c->cfg.sparse_capacity_log2 : 22;
  if (lg < 4 || lg > 30) return fail(c, GPUAGG_EINVAL, "sparse_capacity_log2 %u out of [4,30]", lg);
  const size_t n = (size_t)1 << lg;
  int rc;
  // one interleaved array: slot h = words [5h, 5h + 5) = k0 k1 k2 cnt byt (kSparseSlotWords)
  if ((rc = dev_alloc(c, &c->sv.k0, n * kSparseSlotWords)) || (rc = dev_alloc(c, &c->sv.dropped, 1)) ||
      (rc = dev_alloc(c, &c->d_counter, 1)))
    return rc;
  c->sv.k1 = c->sv.k0 + 1;
  c->sv.k2 = c->sv.k0 + 2;
  c->sv.cnt = c->sv.k0 + 3;
  c->sv.byt = c->sv.k0 + 4;
  c->sv.mask = (uint32_t)(n - 1);
  c->sv.seg_log2 = std::min<uint32_t>(lg, kSparseSegLog2);
  c->sparse_slots = n;
  return GPUAGG_OK;
}

// Slots covered by the dense counters / HLL rows for n interned slots: whole 64-slot
// steps (not powers of two, so the tier-1 kernel's LDS window keeps fitting C2's 10k
// pods), never beyond max_slots.
uint32_t key_cap_for(const gpuagg_ctx *c, size_t n) {
  const size_t cap = std::max<size_t>(64, (n + 63) & ~(size_t)63);
  return (uint32_t)std::min<size_t>(cap, c->cfg.max_slots);
}

// Lays the dense groups out for key_cap slots (hottest group first, see reconcile) and
// sizes the HLL rows.  keep: the accumulated counters / registers move to the new layout
// -- a group's bins are key-major, so its old bins are the prefix of its new ones -- else
// the new state is zero.
int layout_dense(gpuagg_ctx *c, uint32_t key_cap, bool keep) {
  if (keep) {  // the waiting spill lists address the current dense arrays
    if (int rc = fold_pending(c)) return rc;
  } else {
    drop_pending(c);
  }
  uint64_t total = 0;
  std::vector<uint64_t> base(c->groups.size(), 0), old_base(c->groups.size(), 0), old_nbins(c->groups.size(), 0);
  for (size_t g = 0; g < c->groups.size(); ++g) {
    Group &gr = c->groups[g];
    if (gr.sparse) continue;
    old_base[g] = gr.dense_base;
    old_nbins[g] = gr.nkeys * 2 * gr.nsub;
    const uint64_t nkeys = gr.key_mode ? key_cap : 1;
    base[g] = total;
    total += nkeys * 2 * gr.nsub;
  }
  if (total >= (1ull << 32)) return fail(c, GPUAGG_ECAPACITY, "dense counter space >= 2^32 bins");
  HIPCHK(c, x_sync(c, c->stream));
  int rc;
  uint64_t *cnt = nullptr, *byt = nullptr;
  if ((rc = dev_alloc(c, &cnt, total)) || (rc = dev_alloc(c, &byt, total))) {
    dev_free(c, cnt);
    return rc;
  }
  if (total) {
    HIPCHK(c, x_set_async(c, cnt, 0, total * 8, c->stream));
    HIPCHK(c, x_set_async(c, byt, 0, total * 8, c->stream));
  }
  for (size_t g = 0; keep && c->dense_len && g < c->groups.size(); ++g) {
    if (c->groups[g].sparse || !old_nbins[g]) continue;
    const uint64_t nb = std::min<uint64_t>(old_nbins[g], total - base[g]);
    HIPCHK(c, x_copy_async(c, cnt + base[g], c->d_dense_cnt + old_base[g], nb * 8, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, x_copy_async(c, byt + base[g], c->d_dense_byt + old_base[g], nb * 8, hipMemcpyDeviceToDevice, c->stream));
  }
  if (c->cfg.hll_precision) {
    const size_t len = (size_t)key_cap << c->cfg.hll_precision;
    uint8_t *hll = nullptr;
    if ((rc = dev_alloc(c, &hll, len))) {
      dev_free(c, cnt);
      dev_free(c, byt);
      return rc;
    }
    HIPCHK(c, x_set_async(c, hll, 0, len, c->stream));
    if (keep && c->hll_len)
      HIPCHK(c, x_copy_async(c, hll, c->d_hll, std::min(len, c->hll_len), hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, x_sync(c, c->stream));
    dev_free(c, c->d_hll);
    c->d_hll = hll;
    c->hll_len = len;
  }
  HIPCHK(c, x_sync(c, c->stream));
  dev_free(c, c->d_dense_cnt);
  dev_free(c, c->d_dense_byt);
  c->d_dense_cnt = cnt;
  c->d_dense_byt = byt;
  c->dense_len = total;
  for (size_t g = 0; g < c->groups.size(); ++g) {
    Group &gr = c->groups[g];
    if (gr.sparse) continue;
    gr.dense_base = base[g];
    gr.nkeys = gr.key_mode ? key_cap : 1;
    c->plan.g[g].dense_base = base[g];
    c->plan.g[g].nbins = (uint32_t)(gr.nkeys * 2 * gr.nsub);
  }
  c->key_cap = key_cap;
  return GPUAGG_OK;
}

void drain_timing(gpuagg_ctx *c) {
  for (auto &ev : c->pending_events) {
    float ms = 0.f, fold = 0.f;
    if (hipEventSynchronize(ev[2]) == hipSuccess && hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess &&
        hipEventElapsedTime(&fold, ev[1], ev[2]) == hipSuccess) {
      c->stats.kernel_ms += ms;
      c->stats.fold_ms += fold;
      c->stats.kernel_launches += 1;
    }
  }
  // (a chained launch's start is the previous launch's end: each event destroyed once)
  for (size_t i = 0; i < c->pending_events.size(); ++i) {
    const auto &ev = c->pending_events[i];
    if (i == 0 || ev[0] != c->pending_events[i - 1][2]) hipEventDestroy(ev[0]);
    hipEventDestroy(ev[1]);
    hipEventDestroy(ev[2]);
  }
  c->pending_events.clear();
  c->tm_end = nullptr;
  c->tm_chain = false;
  for (auto &ev : c->pending_decode) {
    float ms = 0.f;
    if (hipEventSynchronize(ev[1]) == hipSuccess && hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) {
      c->stats.decode_ms += ms;
      c->stats.decode_launches += 1;
    }
    for (hipEvent_t e : ev) hipEventDestroy(e);
  }
  c->pending_decode.clear();
  for (auto &ev : c->pending_sketch) {
    float ms = 0.f;
    if (hipEventSynchronize(ev[1]) == hipSuccess && hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess)
      c->stats.sketch_ms += ms;
    for (hipEvent_t e : ev) hipEventDestroy(e);
  }
  c->stats.sketch_launches += c->pending_sketch_submits;
  c->pending_sketch_submits = 0;
  c->pending_sketch.clear();
  for (auto &ev : c->pending_fold) {
    float ms = 0.f;
    if (hipEventSynchronize(ev[1]) == hipSuccess && hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess)
      c->stats.fold_ms += ms;
    for (hipEvent_t e : ev) hipEventDestroy(e);
  }
  c->pending_fold.clear();
}

// Count-min windows: 2^15 columns (128 KiB of LDS in the fold); at most 4096 windows
// (16 KiB of scatter counters), else every update is a direct global atomic.
constexpr uint32_t kCmsWindowShift = 15, kCmsMaxWindows = 4096;
// HLL windows: 2^shift source pods whose registers fit 128 KiB of LDS (entries carry the
// pod-in-window in 8 bits and the register index in 18, so p <= 17 and shift <= 8)
constexpr uint32_t kHllWindowLog2Bytes = 17, kHllMaxWindows = 8192;

// Records per scatter workgroup between deferred sketch folds: 8 full-size C3 launches
// (2^27 records over 256 workgroups), 256 of the Go plugin's 2^22-record batches; ~15 GB of
// lists at C3's geometry (d = 4, 256 workgroups), plus the HLL re-bucketing lists at the
// fold.  Each fold rewrites the whole HLL register array and every count-min row, so fewer,
// larger folds pay that once per 8 launches instead of once per 2: C3 step 2.41 -> 2.30 ms
// (2^20 until round 6; 2^21: 2.37; profiles/round6/exp/r6k_c3_sketch_defer_budget_ab.jsonl).
constexpr uint64_t kSketchDeferRecords = 1ull << 22;

// HLL level-2 (split) lists for `records` scatter entries at most: m / (nsup * b2 * nfine)
// per list, +25 % + 64 of headroom (a full list applies the update with the global CAS).
int size_hll_level2(gpuagg_ctx *c, SketchArgs &s, uint64_t records) {
  const uint64_t nfine = (uint64_t)1 << (s.hll_sshift - s.hll_shift);
  const uint64_t mean2 = records / ((uint64_t)s.hll_nsup * s.hll_b2 * nfine);
  const uint64_t cap2 = (mean2 + mean2 / 4 + 64 + 15) & ~15ULL;
  const size_t n2 = (size_t)s.hll_nsup * s.hll_b2 * nfine;
  int rc;
  if ((rc = ensure_buf(c, &c->d_hll_lists2, &c->hll_lists2_alloc, n2 * cap2))) return rc;
  if ((rc = ensure_buf(c, &c->d_hll_counts2, &c->hll_counts2_alloc, n2))) return rc;
  s.hll_cap2 = (uint32_t)cap2;
  s.hll_lists2 = c->d_hll_lists2;
  s.hll_counts2 = c->d_hll_counts2;
  return GPUAGG_OK;
}

// The deferred sketch scatters' lists folded into the count-min rows and HLL registers.
int fold_pending_sketch(gpuagg_ctx *c) {
  if (!c->sk_pend.active) return GPUAGG_OK;
  c->sk_pend.active = false;
  SketchArgs s = c->sk_pend.s;
  s.passes = kSketchFolds;
  s.accum = false;
  int rc;
  if (s.hll_nsup && (rc = size_hll_level2(c, s, c->sk_pend.rpb * s.blocks))) return rc;
  std::array<hipEvent_t, 2> ev{};
  if (c->timing) {
    for (auto &e : ev) HIPCHK(c, hipEventCreateWithFlags(&e, kTimingEventFlags));
    HIPCHK(c, hipEventRecord(ev[0], c->stream));
  }
  ENQ(c);
  ForkJoin fj{};
  if (!c->cpu && (rc = fold_fork_join(c, &fj))) return rc;
  HIPCHK(c, launch_sketch(s, c->stream, nullptr, c->cpu ? nullptr : &fj));
  if (c->timing) {
    HIPCHK(c, hipEventRecord(ev[1], c->stream));
    c->pending_fold.push_back(ev);
  }
  return GPUAGG_OK;
}

// The sketch pass over n records: count-min scatter + fold, HLL direct (SketchArgs).
int launch_sketches(gpuagg_ctx *c, const ColsView &cv, size_t n) {
  int rc;
  SketchArgs s{};
  s.ip_slots = c->d_ip;
  s.ip_mask = (uint32_t)(c->ip_cap ? c->ip_cap / 2 - 1 : 0);  // bucket mask
  s.ip_pre = c->radix ? c->d_rpre : nullptr;
  s.ip_blk = c->radix ? c->d_rblk : nullptr;
  s.ip_seed = c->ip_seed;
  s.cms = c->d_cms;
  s.cms_depth = c->cms_len ? c->cfg.cms_depth : 0;
  s.cms_wlog2 = c->cfg.cms_width_log2;
  s.hll = c->d_hll;
  s.hll_p = c->hll_len ? c->cfg.hll_precision : 0;
  s.blocks = c->n_cu;
  s.win_shift = std::min<uint32_t>(kCmsWindowShift, s.cms_wlog2);
  s.hll_slots = s.hll_p ? (uint32_t)(c->hll_len >> s.hll_p) : 0;
  if (c->cpu) {  // relaxed atomics on the shared rows / registers
    s.cols = ColsView{cv.src_ip, cv.dst_ip, nullptr, cv.meta, cv.ports, nullptr};
    s.n = n;
    c->cpu->sketch(s);
    return GPUAGG_OK;
  }
  if (s.hll_p && c->ipl_all_bytes) {
    s.ipl = c->d_ipl_all;
    s.ipl_nb = c->ipl_all_nb;
    s.ipl_seed = c->ipl_all_seed;
    s.ipl_bytes = c->ipl_all_bytes;
    s.ipl_radix = c->ipl_all_radix;
    s.ipl_dense = c->ipl_all_dense;
    s.ipl_npfx = c->ipl_all_npfx;
    for (uint32_t j = 0; j < kIprMaxPfx; ++j) {
      s.ipl_pfx[j] = c->ipl_all_pfx[j];
      s.ipl_dr[j] = c->ipl_all_dr[j];
    }
  }
  // HLL bucketing: fine windows of 2^hll_shift pods (128 KiB of registers, the fold's
  // LDS), super-windows of 2^hll_sshift pods (~16 of them, the scatter's lists); pod bits
  // of an entry: 26 - p
  uint64_t hnwin = 0, hnsup = 0;
  const bool direct = c->cfg.flags & GPUAGG_FLAG_DIRECT_SKETCH;
  if (!direct && s.hll_p && s.hll_p <= kHllWindowLog2Bytes && s.hll_slots) {
    s.hll_shift = std::min<uint32_t>(8u, kHllWindowLog2Bytes - s.hll_p);
    uint32_t ss = s.hll_shift;
    while ((((uint64_t)s.hll_slots + (1u << ss) - 1) >> ss) > 16 && ss < 26 - s.hll_p && ss < s.hll_shift + 10) ++ss;
    s.hll_sshift = ss;
    hnwin = ((uint64_t)s.hll_slots + (1u << s.hll_shift) - 1) >> s.hll_shift;
    hnsup = ((uint64_t)s.hll_slots + (1u << ss) - 1) >> ss;
    if (hnwin > kHllMaxWindows || hnsup > 1024) hnwin = hnsup = 0;
    s.hll_b2 = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, c->n_cu / std::max<uint64_t>(1, hnsup)));
  }
  const uint64_t nwin = s.cms_depth ? ((uint64_t)s.cms_depth << (s.cms_wlog2 - s.win_shift)) : 0;
  const uint64_t per_launch = (uint64_t)s.blocks << 20;  // <= 2^20 records per scatter workgroup
  // Lists sized for `rpb` records per scatter workgroup (one launch's chunk, or the deferral
  // budget).  CMS: expected entries per list = rpb * depth / nwin, +12.5 % + 2048 of headroom;
  // HLL level 1: at most one entry per record, rpb / nsup per list, +25 % + 64 (a full list
  // falls back to the exact global atomic / CAS).
  auto size_lists = [&](SketchArgs &x, uint64_t rpb) -> int {
    int r;
    x.nwin = 0;
    if (!direct && nwin && nwin <= kCmsMaxWindows) {
      const uint64_t mean = rpb * x.cms_depth / nwin;
      const uint64_t cap = (mean + mean / 8 + 2048 + 7) & ~7ULL;
      if ((r = ensure_buf(c, &c->d_sk_lists, &c->sk_lists_alloc, (size_t)x.blocks * nwin * cap))) return r;
      if ((r = ensure_buf(c, &c->d_sk_counts, &c->sk_counts_alloc, (size_t)x.blocks * nwin))) return r;
      x.nwin = (uint32_t)nwin;
      x.cap = (uint32_t)cap;
      x.lists = c->d_sk_lists;
      x.counts = c->d_sk_counts;
      x.fold_blocks = (uint32_t)nwin * std::max<uint32_t>(1u, c->n_cu / (uint32_t)nwin);
    }
    x.hll_nwin = x.hll_nsup = 0;
    if (hnsup) {
      const uint64_t mean = rpb / hnsup;
      const uint64_t cap = (mean + mean / 4 + 64 + 15) & ~15ULL;
      if ((r = ensure_buf(c, &c->d_hll_lists, &c->hll_lists_alloc, (size_t)x.blocks * hnsup * cap))) return r;
      if ((r = ensure_buf(c, &c->d_hll_counts, &c->hll_counts_alloc, (size_t)x.blocks * hnsup))) return r;
      x.hll_nsup = (uint32_t)hnsup;
      x.hll_nwin = (uint32_t)hnwin;
      x.hll_cap = (uint32_t)cap;
      x.hll_lists = c->d_hll_lists;
      x.hll_counts = c->d_hll_counts;
    }
    return GPUAGG_OK;
  };
  // Timing (gpuagg_set_timing): sketch_ms spans the scatter launches only -- the kernel
  // bench.py names -- and the folds count in fold_ms (fold_pending_sketch, or the pair
  // around a full-size launch's folds below); sketch_launches counts submits.
  auto t_open = [&](std::array<hipEvent_t, 2> &ev) -> int {
    for (auto &e : ev) HIPCHK(c, hipEventCreateWithFlags(&e, kTimingEventFlags));
    HIPCHK(c, hipEventRecord(ev[0], c->stream));
    return GPUAGG_OK;
  };
  auto t_close = [&](std::array<hipEvent_t, 2> &ev, std::vector<std::array<hipEvent_t, 2>> &to) -> int {
    HIPCHK(c, hipEventRecord(ev[1], c->stream));
    to.push_back(ev);
    return GPUAGG_OK;
  };
  if (c->timing) ++c->pending_sketch_submits;
  // Deferred folds (small launches, e.g. the Go plugin's 2^20 records: chunk 4096): the
  // folds' fixed passes -- every count-min row and the whole HLL register array (164 MB at
  // C3's 10k pods, p = 14) are read and rewritten -- cost ~20x the scatter of such a launch,
  // so launches keep appending to one set of lists sized for kSketchDeferRecords records per
  // workgroup and fold_pending folds them once (gpuagg_sync, state reads, merge, relayout,
  // or when the next launch would not fit).
  const uint64_t chunk1 = ((std::min<uint64_t>(n, per_launch) + s.blocks - 1) / s.blocks + 3) & ~3ULL;
  const bool defer = c->defer_folds && !direct && n <= per_launch && 2 * chunk1 <= kSketchDeferRecords &&
                     (nwin || hnsup);
  if (c->sk_pend.active) {
    const SketchArgs &q = c->sk_pend.s;
    const bool fits = defer && c->sk_pend.rpb + chunk1 <= c->sk_pend.budget && q.blocks == s.blocks &&
                      q.cms == s.cms && q.hll == s.hll && q.hll_slots == s.hll_slots &&
                      q.hll_shift == s.hll_shift && q.hll_sshift == s.hll_sshift && q.hll_b2 == s.hll_b2 &&
                      q.lists == c->d_sk_lists && q.hll_lists == c->d_hll_lists;
    if (!fits && (rc = fold_pending_sketch(c))) return rc;
  }
  for (uint64_t off = 0; off < n; off += per_launch) {
    const uint64_t m = std::min<uint64_t>(per_launch, n - off);
    s.cols = ColsView{cv.src_ip + off, cv.dst_ip + off, nullptr, cv.meta + off,
                      cv.ports ? cv.ports + off : nullptr, nullptr};
    s.n = m;
    s.chunk = ((m + s.blocks - 1) / s.blocks + 3) & ~3ULL;  // whole 4-record vectors
    if (defer) {
      const bool accum = c->sk_pend.active;
      if (accum) {  // the waiting lists' geometry
        const SketchArgs &q = c->sk_pend.s;
        s.nwin = q.nwin;
        s.cap = q.cap;
        s.lists = q.lists;
        s.counts = q.counts;
        s.fold_blocks = q.fold_blocks;
        s.hll_nsup = q.hll_nsup;
        s.hll_nwin = q.hll_nwin;
        s.hll_cap = q.hll_cap;
        s.hll_lists = q.hll_lists;
        s.hll_counts = q.hll_counts;
      } else if ((rc = size_lists(s, kSketchDeferRecords))) {
        return rc;
      }
      s.passes = kSketchScatter;
      s.accum = accum;
      ENQ(c);
      std::array<hipEvent_t, 2> ev{};
      if (c->timing && (rc = t_open(ev))) return rc;
      HIPCHK(c, launch_sketch(s, c->stream, &c->sketch_kernel_name));
      if (c->timing && (rc = t_close(ev, c->pending_sketch))) return rc;
      c->sk_pend.rpb = (accum ? c->sk_pend.rpb : 0) + s.chunk;
      c->sk_pend.budget = kSketchDeferRecords;
      c->sk_pend.s = s;
      c->sk_pend.active = true;
      continue;
    }
    if ((rc = size_lists(s, s.chunk))) return rc;
    if (hnsup && (rc = size_hll_level2(c, s, m))) return rc;
    // the scatter, then its folds (kSketchBoth as two calls, so each is timed on its own)
    s.accum = false;
    ENQ(c);
    std::array<hipEvent_t, 2> ev{}, evf{};
    s.passes = kSketchScatter;
    if (c->timing && (rc = t_open(ev))) return rc;
    HIPCHK(c, launch_sketch(s, c->stream, &c->sketch_kernel_name));
    if (c->timing && (rc = t_close(ev, c->pending_sketch))) return rc;
    s.passes = kSketchFolds;
    if (c->timing && (rc = t_open(evf))) return rc;
    HIPCHK(c, launch_sketch(s, c->stream, nullptr));
    if (c->timing && (rc = t_close(evf, c->pending_fold))) return rc;
  }
  return GPUAGG_OK;
}


// Latency state: `full` (reconcile) also drops the clock and the pending requests;
// otherwise (epoch reset after a merge) only the histograms and no_response restart.
int lat_reset(gpuagg_ctx *c, bool full) {
  if (full) {
    c->lat_pend.active = false;  // a new TTL cache: the last batch's decision no longer matters
  } else if (int rc = lat_resolve(c)) {
    return rc;
  }
  if (!c->d_lat) {
    if (!c->lat_enabled) return GPUAGG_OK;
    if (int rc = dev_alloc(c, &c->d_lat, kLatStateWords)) return rc;
    full = true;
  }
  if (full) {
    HIPCHK(c, x_set_async(c, c->d_lat, 0, kLatStateWords * 8, c->stream));
    c->lat_carry_bound = 0;
    c->lat_peak_pending = 0;
    if (c->cpu) c->cpu->latency_reset();
  } else {
    HIPCHK(c, x_set_async(c, c->d_lat + kLatHist, 0, (kLatStateWords - kLatHist) * 8, c->stream));
  }
  return GPUAGG_OK;
}

// The batch in event order when the capacity binds: the ttlcache itself (every event
// depends on the live set the earlier ones left), replayed on the host, where the item
// table (2x LIMIT slots) and the pool stay in cache -- on the GPU this was one thread
// chasing global memory, 1.7 s per 2^20-record batch (profiles/round5/r5l_lat_serial.jsonl).
// Items live in a pool, a linear-probing table maps keys to them (backward-shift
// deletion), and a queue of touches in order is the LRU list (a record is stale once its
// item is touched again or freed): its front valid item is the least recently touched,
// which is also the first to expire.  Reads the events (carried entries at [0, pend), in
// LRU order by a.carry_order) and the state words, writes back the state and the
// carry-out (lat_finish_kernel then advances the clock and the pending count).
int lat_serial_host(gpuagg_ctx *c, const LatArgs &a, uint64_t n, uint64_t pend) {
  std::vector<LatEvent> ev(n);
  std::vector<uint32_t> order(pend);
  unsigned long long st[kLatStateWords];
  HIPCHK(c, x_copy_async(c, ev.data(), a.ev, n * sizeof(LatEvent), hipMemcpyDeviceToHost, c->stream));
  if (pend)
    HIPCHK(c, x_copy_async(c, order.data(), a.carry_order, pend * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, x_copy_async(c, st, a.state, sizeof st, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, x_sync(c, c->stream));
  const uint32_t enabled = c->lat_enabled;
  uint32_t tsize = 1024;
  while (tsize < 2 * a.limit) tsize <<= 1;
  const uint32_t mask = tsize - 1;
  std::vector<uint32_t> table(tsize, 0u);  // pool index + 1 (0: empty)
  std::vector<LatEntry> pool;
  pool.reserve(std::min<uint64_t>(a.limit, n));
  std::vector<uint32_t> free_idx;
  std::vector<LatTouch> queue;
  queue.reserve(n);
  size_t qh = 0;
  uint64_t live = 0;
  auto home = [&](uint64_t k0, uint64_t k1) { return (uint32_t)fmix64(k0 ^ fmix64(k1 ^ 0x6A09E667F3BCC909ULL)) & mask; };
  auto find = [&](uint64_t k0, uint64_t k1) -> int64_t {  // table slot, or -1
    for (uint32_t s = home(k0, k1);; s = (s + 1) & mask) {
      const uint32_t v = table[s];
      if (!v) return -1;
      const LatEntry &x = pool[v - 1];
      if (x.k0 == k0 && x.k1 == k1) return s;
    }
  };
  auto erase = [&](uint32_t s) {  // backward-shift deletion, frees the item
    const uint32_t idx = table[s] - 1;
    pool[idx].seq = ~0ULL;
    free_idx.push_back(idx);
    for (uint32_t t = (s + 1) & mask;; t = (t + 1) & mask) {
      const uint32_t v = table[t];
      if (!v) break;
      const uint32_t hm = home(pool[v - 1].k0, pool[v - 1].k1);
      // the item at t may move to s unless its home lies cyclically in (s, t]
      const bool stay = s <= t ? (hm > s && hm <= t) : (hm > s || hm <= t);
      if (!stay) {
        table[s] = v;
        s = t;
      }
    }
    table[s] = 0u;
    --live;
  };
  auto insert = [&](const LatEntry &x) {
    uint32_t idx;
    if (!free_idx.empty()) {
      idx = free_idx.back();
      free_idx.pop_back();
      pool[idx] = x;
    } else {
      idx = (uint32_t)pool.size();
      pool.push_back(x);
    }
    uint32_t s = home(x.k0, x.k1);
    while (table[s]) s = (s + 1) & mask;
    table[s] = idx + 1;
    queue.push_back(LatTouch{x.seq, idx, 0u});
    ++live;
  };
  auto front = [&]() -> uint32_t {  // the front valid item (skipping stale records), or ~0
    while (qh < queue.size()) {
      const LatTouch r = queue[qh];
      if (pool[r.idx].seq == r.seq) return r.idx;
      ++qh;
    }
    return ~0u;
  };
  auto bucket = [](int64_t v) -> uint32_t { return v <= 0 ? 0u : v >= 5 ? 10u : (uint32_t)(2 * v); };
  for (uint64_t k = 0; k < pend; ++k) {  // carried items, least recently touched first
    const LatEvent &e = ev[order[k]];
    insert(LatEntry{e.k0, e.k1, e.clock, e.seq, e.nanos, (e.bits >> 2) & 1u});
  }
  for (uint64_t pos = pend; pos < n; ++pos) {
    const LatEvent e = ev[pos];
    for (uint32_t f = front(); f != ~0u && e.clock > pool[f].expires; f = front()) {
      erase((uint32_t)find(pool[f].k0, pool[f].k1));  // expired before this record
      ++qh;
      if (enabled & 4u) st[kLatNoResponse] += 1;
    }
    const int64_t s = find(e.k0, e.k1);
    if ((e.bits & 3u) == 1u) {  // request
      if (s >= 0) {  // Get hit: touched
        const uint32_t idx = table[s] - 1;
        pool[idx].expires = e.clock + kLatTtlNs;
        pool[idx].seq = e.seq;
        queue.push_back(LatTouch{e.seq, idx, 0u});
        continue;
      }
      if (live >= a.limit) {  // Set at capacity: the LRU back goes, uncounted
        const uint32_t f = front();
        erase((uint32_t)find(pool[f].k0, pool[f].k1));
        ++qh;
        st[kLatCapEvictions] += 1;
      }
      insert(LatEntry{e.k0, e.k1, e.clock + kLatTtlNs, e.seq, e.nanos, (e.bits >> 2) & 1u});
    } else if (s >= 0) {  // reply: latency, then Delete
      const LatEntry x = pool[table[s] - 1];
      const int64_t d = (int64_t)e.nanos - (int64_t)x.nanos;
      const int64_t ad = d < 0 ? -d : d;
      const int64_t lat = (d < 0 ? -1 : 1) * ((ad + 500000) / 1000000);  // math.Round
      const uint32_t bk = bucket(lat);
      if (enabled & 1u) {
        st[kLatHist + bk] += 1;
        st[kLatHist + 11] += 1;
        st[kLatHist + 12] += (unsigned long long)lat;
      }
      if ((enabled & 2u) && x.syn && ((e.bits >> 2) & 1u) && ((e.bits >> 3) & 1u)) {
        st[kLatHandshake + bk] += 1;
        st[kLatHandshake + 11] += 1;
        st[kLatHandshake + 12] += (unsigned long long)lat;
      }
      erase((uint32_t)s);
    }
  }
  // batch end: expired items count, the rest carry over in LRU order
  const unsigned long long clk_end = st[kLatClockEnd];
  std::vector<LatEvent> out;
  for (uint32_t f = front(); f != ~0u; f = front()) {
    const LatEntry x = pool[f];
    if (clk_end > x.expires) {
      if (enabled & 4u) st[kLatNoResponse] += 1;
    } else {
      out.push_back(LatEvent{x.k0, x.k1, x.expires, x.seq, x.nanos, 3u | (x.syn ? 4u : 0u)});
    }
    pool[f].seq = ~0ULL;
    ++qh;
  }
  st[kLatCarryOut] = out.size();
  st[kLatCapBatches] += 1;
  if (!out.empty())
    HIPCHK(c, x_copy_async(c, a.carry_out, out.data(), out.size() * sizeof(LatEvent), hipMemcpyHostToDevice,
                           c->stream));
  HIPCHK(c, x_copy_async(c, a.state, st, sizeof st, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, x_sync(c, c->stream));  // the host buffers go out of scope
  return GPUAGG_OK;
}

// The TTL join over one batch (see gpuagg_latency.hip); waits for the event count.
int launch_latency(gpuagg_ctx *c, const ColsView &cv, size_t n) {
  int rc;
  if (!cv.ports || !cv.tcp_id || !cv.time_ns)
    return fail(c, GPUAGG_EINVAL, "node-apiserver latency metrics read the ports, tcp_id and time_ns columns");
  if (!c->d_lat && (rc = lat_reset(c, true))) return rc;
  if ((rc = lat_resolve(c))) return rc;  // the previous batch first (its events are still in place)
  if (c->cpu) {  // the TTL join in record order on the host
    LatArgs a{};
    a.src = cv.src_ip;
    a.dst = cv.dst_ip;
    a.meta = cv.meta;
    a.ports = cv.ports;
    a.tcp_id = cv.tcp_id;
    a.time_ns = cv.time_ns;
    a.n = n;
    a.api = c->d_api;
    a.n_api = (uint32_t)c->api_ips.size();
    a.state = c->d_lat;
    a.limit = c->cfg.latency_limit ? c->cfg.latency_limit : kLatLimit;
    c->lat_peak_pending = std::max<uint64_t>(c->lat_peak_pending, c->d_lat[kLatPending]);
    c->cpu->latency(a, c->lat_enabled);
    return GPUAGG_OK;
  }
  LatArgs a{};
  a.src = cv.src_ip;
  a.dst = cv.dst_ip;
  a.meta = cv.meta;
  a.ports = cv.ports;
  a.tcp_id = cv.tcp_id;
  a.time_ns = cv.time_ns;
  a.n = n;
  // units: one wave over >= 8192 contiguous rows (16 waves per CU at 100M rows; the
  // one-workgroup scan reads a dozen units per thread)
  a.blocks = (uint32_t)std::min<uint64_t>(kLatMaxUnits, (n + 8191) / 8192);
  a.chunk = ((n + a.blocks - 1) / a.blocks + 3) & ~3ULL;
  a.vec = (((uintptr_t)cv.meta | (uintptr_t)cv.tcp_id | (uintptr_t)cv.time_ns) & 15u) == 0;
  a.api = c->d_api;
  a.n_api = (uint32_t)c->api_ips.size();
  a.state = c->d_lat;
  if ((rc = ensure_buf(c, &c->d_lat_blk_cnt, &c->lat_blk_alloc, a.blocks))) return rc;
  if (!c->d_lat_blk_max) {
    const size_t nb = kLatMaxUnits;
    if ((rc = dev_alloc(c, &c->d_lat_blk_max, nb)) || (rc = dev_alloc(c, &c->d_lat_blk_clk, nb)) ||
        (rc = dev_alloc(c, &c->d_lat_blk_base, nb)))
      return rc;
    if (c->lat_blk_alloc < nb) {  // keep every per-block array the same size
      dev_free(c, c->d_lat_blk_cnt);
      c->lat_blk_alloc = 0;
      if ((rc = ensure_buf(c, &c->d_lat_blk_cnt, &c->lat_blk_alloc, nb))) return rc;
    }
  }
  a.blk_cnt = c->d_lat_blk_cnt;
  a.blk_max = c->d_lat_blk_max;
  a.blk_clk = c->d_lat_blk_clk;
  a.blk_base = c->d_lat_blk_base;
  // events: carried entries + at most one per record
  const size_t cap = c->lat_carry_bound + n;
  if (cap > c->lat_ev_alloc) {
    HIPCHK(c, x_sync(c, c->stream));
    dev_free(c, c->d_lat_ev);
    dev_free(c, c->d_lat_hash);
    dev_free(c, c->d_lat_idx);
    dev_free(c, c->d_lat_delta);
    c->lat_ev_alloc = 0;
    if ((rc = dev_alloc(c, &c->d_lat_ev, cap)) || (rc = dev_alloc(c, &c->d_lat_hash, 2 * cap)) ||
        (rc = dev_alloc(c, &c->d_lat_idx, 2 * cap)) || (rc = dev_alloc(c, &c->d_lat_delta, 2 * (cap + 1))))
      return rc;
    c->lat_ev_alloc = cap;
  }
  a.limit = c->cfg.latency_limit ? c->cfg.latency_limit : kLatLimit;
  if (!c->d_lat_max_live && (rc = dev_alloc(c, &c->d_lat_max_live, 1))) return rc;
  a.delta = c->d_lat_delta;
  a.live = c->d_lat_delta + c->lat_ev_alloc + 1;
  a.max_live = c->d_lat_max_live;
  a.ev = c->d_lat_ev;
  a.hash_in = c->d_lat_hash;
  a.hash_out = c->d_lat_hash + c->lat_ev_alloc;
  a.idx_in = c->d_lat_idx;
  a.idx_out = c->d_lat_idx + c->lat_ev_alloc;
  constexpr size_t kLatReadWords = kLatEvents - kLatPending + 1;
  if (!c->h_lat_n && hipHostMalloc((void **)&c->h_lat_n, 8 * (kLatReadWords + 1), hipHostMallocDefault) != hipSuccess)
    return fail(c, GPUAGG_ENOMEM, "hipHostMalloc(%zu)", 8 * (kLatReadWords + 1));
  a.carry_in = c->d_lat_carry[c->lat_carry_cur];  // copied into the events by the front
  ENQ(c);
  HIPCHK(c, launch_latency_front(a, c->stream));
  HIPCHK(c, x_copy_async(c, c->h_lat_n, c->d_lat + kLatPending, 8 * kLatReadWords, hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, x_sync(c, c->stream));
  const uint64_t ne = c->h_lat_n[kLatEvents - kLatPending];
  c->lat_peak_pending = std::max<uint64_t>(c->lat_peak_pending, c->h_lat_n[0]);  // carried into this batch
  // carry-out buffer: at most one entry per event
  if (ne > c->lat_carry_alloc) {
    LatEvent *keep = c->d_lat_carry[c->lat_carry_cur];  // read by this batch already (copied)
    dev_free(c, c->d_lat_carry[c->lat_carry_cur ^ 1]);
    c->d_lat_carry[c->lat_carry_cur] = nullptr;
    dev_free(c, keep);
    c->lat_carry_alloc = 0;
    if ((rc = dev_alloc(c, &c->d_lat_carry[0], ne)) || (rc = dev_alloc(c, &c->d_lat_carry[1], ne))) return rc;
    c->lat_carry_alloc = ne;
  }
  a.carry_out = c->d_lat_carry[c->lat_carry_cur ^ 1];
  size_t tb = 0;
  HIPCHK(c, latency_sort_bytes(ne, &tb));
  if (tb > c->lat_tmp_alloc) {
    if (c->d_lat_tmp) hipFree(c->d_lat_tmp);
    c->d_lat_tmp = nullptr;
    c->lat_tmp_alloc = 0;
    HIPCHK(c, hipMalloc(&c->d_lat_tmp, tb));
    c->lat_tmp_alloc = tb;
  }
  // the carried entries' LRU order (by last touch), read by the sequential pass if the
  // capacity binds; they sit at event positions [0, pending)
  const uint64_t pend = c->h_lat_n[0];
  if (pend) {
    if (pend > c->lat_order_alloc) {
      dev_free(c, c->d_lat_okeys);
      dev_free(c, c->d_lat_ovals);
      c->lat_order_alloc = 0;
      if ((rc = dev_alloc(c, &c->d_lat_okeys, 2 * pend)) || (rc = dev_alloc(c, &c->d_lat_ovals, 2 * pend))) return rc;
      c->lat_order_alloc = pend;
    }
    HIPCHK(c, latency_carry_order(a.ev, pend, c->d_lat_okeys, c->d_lat_ovals, c->d_lat_tmp, c->lat_tmp_alloc,
                                  c->stream));
    a.carry_order = c->d_lat_ovals + pend;
  }
  HIPCHK(c, launch_latency_check(a, ne, c->d_lat_tmp, c->lat_tmp_alloc, c->lat_enabled, c->stream));
  // The one decision the host takes -- does the capacity bind in this batch? -- is not
  // waited for here (a second blocking sync per batch undid the async submit).
  // The parallel walk and the finish run guarded on the device (both return at once when
  // the live-count maximum exceeds the limit), the maximum comes back into pinned memory
  // behind them, and lat_resolve -- at the next batch, sync, state read, merge or epoch
  // reset, before anything touches this batch's events -- replays a bound batch on the
  // host (in event order, as the ttlcache) and finishes it then.
  c->h_lat_n[kLatReadWords] = 0;
  if (ne) {
    HIPCHK(c, launch_latency_walk(a, ne, c->lat_enabled, c->stream));
    HIPCHK(c, x_copy_async(c, &c->h_lat_n[kLatReadWords], c->d_lat_max_live, 4, hipMemcpyDeviceToHost,
                           c->stream));
  }
  HIPCHK(c, launch_latency_finish(a, ne, true, c->stream));
  c->lat_pend.active = ne != 0;
  c->lat_pend.a = a;
  c->lat_pend.ne = ne;
  c->lat_pend.pend = pend;
  c->lat_carry_cur ^= 1;
  c->lat_carry_bound = ne;
  return GPUAGG_OK;
}

// The last latency batch's capacity decision (launch_latency): a batch whose live count
// passed the limit is replayed on the host and finished.  Nothing between that batch and
// this call wrote its events, order keys or state words (the next batch calls this first).
int lat_resolve(gpuagg_ctx *c) {
  if (!c->lat_pend.active) return GPUAGG_OK;
  c->lat_pend.active = false;
  constexpr size_t kLatReadWords = kLatEvents - kLatPending + 1;
  HIPCHK(c, x_sync(c, c->stream));
  const int32_t max_live = (int32_t)(uint32_t)c->h_lat_n[kLatReadWords];
  const LatArgs &a = c->lat_pend.a;
  if ((uint64_t)(int64_t)max_live <= a.limit) return GPUAGG_OK;  // walked and finished on the device
  int rc = lat_serial_host(c, a, c->lat_pend.ne, c->lat_pend.pend);
  if (rc) return rc;
  HIPCHK(c, launch_latency_finish(a, c->lat_pend.ne, false, c->stream));
  return GPUAGG_OK;
}

// Launches whose list folds may wait for one fold_pending (see Pending).
constexpr uint64_t kDeferLaunches = 64;
// Spill-only plans defer their folds at launches of at most this many records per workgroup
// (the Go plugin's 2^22-record batches: 2^14; full-size launches fold per batch, see launch()).
constexpr uint64_t kSmallLaunchChunk = 1ull << 16;
// Default device memory for the wide-key segment lists of one ctx (32-byte entries;
// gpuagg_config.wide_list_mib overrides it): 32 GiB (1024 entries per workgroup and segment at 2^24
// slots), at most 1/8 of the device.  A list that fills sends its updates to memory-side
// atomics, and under C4's skew 8 GiB (256 entries) overflowed within one launch: 1.74 ->
// 1.32 ms per 100M records (profiles/round3/exp/v2_wide_list_bytes.jsonl).
constexpr uint64_t kWideListBytes = 32ull << 30;

int launch(gpuagg_ctx *c, const ColsView &cv, size_t n) {
  int rc = 0;
  if (n == 0) return GPUAGG_OK;
  if (!c->ip_cap) return fail(c, GPUAGG_ESTATE, "gpuagg_set_endpoints was never called");
  if (c->plan.need_ports && !cv.ports) return fail(c, GPUAGG_EINVAL, "enabled metrics read the ports column");
  if ((c->cms_len) && !cv.ports) return fail(c, GPUAGG_EINVAL, "count-min reads the ports column");
  if (c->plan.need_dns && !cv.dns_id) return fail(c, GPUAGG_EINVAL, "enabled DNS metrics read the dns_id column");
  LaunchArgs a{};
  a.ip_slots = c->d_ip;
  a.ip_mask = (uint32_t)(c->ip_cap / 2 - 1);  // bucket mask
  a.ip_pre = c->radix ? c->d_rpre : nullptr;
  a.ip_blk = c->radix ? c->d_rblk : nullptr;
  a.ip_rpn = c->radix && c->radix_n <= kRadixSmall ? c->radix_n : 0u;
  for (uint32_t j = 0; j < kRadixSmall / 2; ++j) a.ip_rp[j] = c->radix_pfx[j];
  a.ip_seed = c->ip_seed;
  a.plan = c->plan;
  a.dense_cnt = c->d_dense_cnt;
  a.dense_byt = c->d_dense_byt;
  a.dense_len = c->dense_len;
  a.sparse = c->sv;
  a.cms = c->d_cms;
  a.cms_depth = c->cms_len ? c->cfg.cms_depth : 0;
  a.cms_wlog2 = c->cfg.cms_width_log2;
  a.hll = c->d_hll;
  a.hll_p = c->hll_len ? c->cfg.hll_precision : 0;
  // sketches run in their own pass (launch_sketches) so the metric groups keep the
  // dense fast paths
  a.cms_depth = 0;
  a.hll_p = 0;
  // dense local-context fast path: every group dense, no sketches
  a.dense_ng = 0;
  a.dns_compact = false;
  if (c->plan.local && c->plan.ngroups > 0 && !a.cms_depth && !a.hll_p) {
    // every group dense, or -- compact plan -- dense and DNS (keys of 64 bits, inserted
    // through the segment lists by the dense kernel)
    bool all_dense = true;
    for (int g = 0; g < c->plan.ngroups; ++g) {
      const bool dns = c->plan.g[g].family == FAM_DNS_REQ || c->plan.g[g].family == FAM_DNS_RESP;
      if (c->plan.g[g].sparse && c->sv.compact && dns && c->sparse_slots &&
          (c->sparse_slots >> c->sv.seg_log2) <= kSparseMaxSegLists && !(c->cfg.flags & GPUAGG_FLAG_DIRECT_SKETCH))
        a.dns_compact = true;
      else
        all_dense &= !c->plan.g[g].sparse;
    }
    if (!all_dense) a.dns_compact = false;
    if (all_dense)
      for (uint32_t ng : {1u, 2u, 4u, 8u})
        if ((uint32_t)c->plan.ngroups <= ng) {
          a.dense_ng = ng;
          break;
        }
  }
  if (c->cpu) {  // host threads: every update direct (no LDS, lists or spill)
    a.cols = cv;
    a.n = n;
    const auto t0 = std::chrono::steady_clock::now();
    if (c->plan.ngroups > 0) c->cpu->aggregate(a);
    if (c->host_timing) {
      c->stats.kernel_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      c->stats.kernel_launches += 1;
    }
    c->kernel_name = "cpu";
    if ((c->cms_len || c->hll_len) && (rc = launch_sketches(c, cv, n))) return rc;
    if (c->lat_enabled && (rc = launch_latency(c, cv, n))) return rc;
    c->stats.records += n;
    c->stats.batches += 1;
    c->stats.last_kernel = GPUAGG_KERNEL_CPU;
    return GPUAGG_OK;
  }
  // geometry: one 1024-thread workgroup per CU holding L dense bins in LDS
  // LDS window: the longest prefix of whole dense groups (hottest first) that fits
  std::vector<std::pair<uint64_t, uint64_t>> spans;  // (base, bins) of dense groups
  for (int g = 0; g < c->plan.ngroups; ++g)
    if (!c->plan.g[g].sparse) spans.emplace_back(c->plan.g[g].dense_base, c->plan.g[g].nbins);
  std::sort(spans.begin(), spans.end());
  auto prefix = [&](uint64_t limit) {
    uint32_t L = 0;
    for (auto &sp : spans) {
      if (sp.first != L || sp.first + sp.second > limit) break;
      L = (uint32_t)(sp.first + sp.second);
    }
    return L;
  };
  // compact group-by keys (generic kernel) go through per-segment lists whose fill
  // counters take LDS words from the dense window
  const bool generic = !a.dense_ng || a.dns_compact;  // kernels that take compact-key lists
  const uint64_t sp_nwin = c->sparse_slots ? c->sparse_slots >> c->sv.seg_log2 : 0;
  // wide (192-bit) keys take per-segment lists too when the table has at most 4096
  // segments of 2^12 slots (sparse_fold_wide_kernel folds one per workgroup)
  const bool wide_lists = !c->sv.compact && c->sparse_slots && c->sparse_slots <= (1ull << kWideMaxLog2) &&
                          !(c->cfg.flags & GPUAGG_FLAG_NO_WIDE_LISTS);
  const bool sp_lists = generic && (c->sv.compact || wide_lists) && sp_nwin && sp_nwin <= kSparseMaxSegLists &&
                        !(c->cfg.flags & GPUAGG_FLAG_DIRECT_SKETCH);
  // plans with HBM-table keys (remote context, ip / port options): an LDS cache of the
  // hot keys per workgroup in front of the table (hot_add in gpuagg_kernels.hip)
  const bool hot = generic && c->sparse_slots && !c->sv.compact && !(c->cfg.flags & GPUAGG_FLAG_NO_HOT_KEYS);
  a.hot_n = hot ? kHotKeys : 0u;
  a.lds_bins = prefix(kLdsMaxBins - (sp_lists ? (uint32_t)(sp_nwin + 1) / 2 : 0u) -
                      (hot ? kHotKeys * kHotKeyBytes / 8 + 1 : 0u));
  // tier-1: the LDS IP image plus u32 bins, when at least the hottest group fits
  a.tier1 = false;
  a.sig = 0;
  if (a.dense_ng && a.dns_compact && c->plan.ngroups <= 8) {  // dense_local_kernel's signature
    uint32_t sig = 0;
    for (int g = 0; g < c->plan.ngroups; ++g)
      sig |= sig_group(c->plan.g[g].family, !c->plan.g[g].sparse &&
                                                c->plan.g[g].dense_base + c->plan.g[g].nbins <= a.lds_bins)
             << (4 * g);
    a.sig = sig;
  }
  if (a.dense_ng && !a.dns_compact && c->ipl_bytes && !spans.empty() &&
      c->ipl_bytes + kL4ExtraBytes < kLdsBytes) {
    // (with no group in LDS every update spills, but the IP probes still stay on-chip)
    const uint32_t L4 = prefix((kLdsBytes - c->ipl_bytes - kL4ExtraBytes) / 4);
    {
      a.tier1 = true;
      a.lds_bins = L4;
      a.sig = 0;
      if (c->plan.ngroups <= 8) {  // groups in layout order, as the kernel indexes them
        uint32_t sig = 0;
        for (int g = 0; g < c->plan.ngroups; ++g)
          sig |= sig_group(c->plan.g[g].family, c->plan.g[g].dense_base + c->plan.g[g].nbins <= L4)
                 << (4 * g);
        a.sig = sig;
      }
      a.ipl = c->d_ipl;
      a.ipl_nb = c->ipl_nb;
      a.ipl_seed = c->ipl_seed;
      a.ipl_bytes = c->ipl_bytes;
      a.ipl_radix = c->ipl_radix;
      a.ipl_dense = c->ipl_dense;
      a.ipl_npfx = c->ipl_npfx;
      for (uint32_t j = 0; j < kIprMaxPfx; ++j) {
        a.ipl_pfx[j] = c->ipl_pfx[j];
        a.ipl_dr[j] = c->ipl_dr[j];
      }
    }
  }
  // remote context on the wide-key path: the LDS image of every pod IP (wide_kernel takes
  // it when it fits next to the hot-key cache; the context never reads the apiserver flag)
  if (hot && c->remote && !a.tier1 && c->ipl_all_bytes) {
    a.ipl = c->d_ipl_all;
    a.ipl_nb = c->ipl_all_nb;
    a.ipl_seed = c->ipl_all_seed;
    a.ipl_bytes = c->ipl_all_bytes;
    a.ipl_radix = c->ipl_all_radix;
    a.ipl_dense = c->ipl_all_dense;
    a.ipl_npfx = c->ipl_all_npfx;
    for (uint32_t j = 0; j < kIprMaxPfx; ++j) {
      a.ipl_pfx[j] = c->ipl_all_pfx[j];
      a.ipl_dr[j] = c->ipl_all_dr[j];
    }
  }
  // one 1024-thread workgroup per CU whenever LDS holds bins or spill counters: with
  // dense bins but no LDS prefix (C5: 100k-pod groups) 4x fewer workgroups mean 4x
  // fewer, longer spill lists for the fold (same 16 waves per CU)
  // (the hot-key cache alone fills ~2/3 of the LDS: with 256-thread workgroups a CU would
  // run 4 waves)
  const bool wide = a.lds_bins || a.tier1 || c->dense_len > 0 || a.hot_n;
  a.blocks = wide ? c->n_cu : c->n_cu * 4;
  a.threads = wide ? 1024 : 256;
  const uint64_t per_launch = (uint64_t)a.blocks * kMaxRecordsPerBlock;
  for (uint64_t off = 0; c->plan.ngroups > 0 && off < n; off += per_launch) {
    const uint64_t m = std::min<uint64_t>(per_launch, n - off);
    auto sh = [off](const uint32_t *p) { return p ? p + off : nullptr; };
    a.cols = ColsView{sh(cv.src_ip), sh(cv.dst_ip), sh(cv.bytes), sh(cv.meta), sh(cv.ports), sh(cv.dns_id)};
    a.n = m;
    a.chunk = ((m + a.blocks - 1) / a.blocks + 3) & ~3ULL;
    if (hot) {
      // the cache is flushed into the lists once per workgroup and launch: at small batches
      // (the Go plugin's 1M records: 4k per workgroup) a full 2048-entry cache doubled the
      // appends, so it is sized ~chunk / 8 (256 .. kHotKeys entries; under Zipf(1.2) the
      // top 256 keys still carry ~70 % of the updates)
      uint32_t hn = 256;
      while (hn < kHotKeys && (uint64_t)hn * 16 <= a.chunk) hn <<= 1;
      a.hot_n = hn;
    }
    auto al = [](const uint32_t *p) { return ((uintptr_t)p & 15u) == 0; };
    a.vec = al(a.cols.src_ip) && al(a.cols.dst_ip) && al(a.cols.bytes) && al(a.cols.meta) &&
            (!(c->plan.need_ports || c->cms_len) || al(a.cols.ports)) &&
            (!c->plan.need_dns || al(a.cols.dns_id));
    a.spill = nullptr;
    a.spill_count = nullptr;
    a.nwin = 0;
    a.stage_b = nullptr;
    a.stage_a = nullptr;
    if (a.tier1 && a.lds_bins) {  // per-workgroup copies of the LDS bins, summed after
      a.stage_a_stride = (a.lds_bins + 3u) & ~3u;
      // accumulating copies are summed before their buffer can be reallocated
      if (c->pend.active && c->pend.a.stage_defer && (size_t)a.blocks * a.stage_a_stride > c->stage_a_alloc &&
          (rc = fold_pending_dense(c)))
        return rc;
      if ((rc = ensure_buf(c, &c->d_stage_a, &c->stage_a_alloc, (size_t)a.blocks * a.stage_a_stride)))
        return rc;
      a.stage_a = c->d_stage_a;
    }
    // List geometry for `budget` records per workgroup: spill lists per fold window for
    // the bins past the LDS window (overflow falls back to global atomics; a multiple of 4
    // keeps lists 16-byte aligned), compact-key lists per table segment (at most one
    // insert per record, hashed evenly: budget / nwin per list + 25 % + 64; a full list
    // inserts in place, exact).
    struct Geom {
      uint32_t nwin = 0, spill_cap = 0, win_blocks = 0, sp_nwin = 0, sp_cap = 0, win_shift = 0;
      bool operator==(const Geom &o) const {
        return nwin == o.nwin && spill_cap == o.spill_cap && win_blocks == o.win_blocks && sp_nwin == o.sp_nwin &&
               sp_cap == o.sp_cap && win_shift == o.win_shift;
      }
    };
    const uint32_t list_words = c->sv.compact ? 1u : (c->sv.narrow ? kWideNarrowWords : kWideEntryWords);
    auto geom = [&](uint64_t budget) {
      Geom g;
      if (c->dense_len > a.lds_bins) {
        const uint64_t rem = c->dense_len - a.lds_bins;
        const uint32_t shift = kFoldWindowShift;
        const uint32_t nwin = (uint32_t)((rem + (1ull << shift) - 1) >> shift);
        const uint64_t cap = ((2 * budget / nwin + 4096) + 3) & ~3ULL;
        if (nwin <= kMaxSpillWindows && cap < (1u << 24)) {  // 24-bit index math in the kernels
          g.nwin = nwin;
          g.win_shift = shift;
          g.spill_cap = (uint32_t)cap;
          g.win_blocks = nwin * std::max<uint32_t>(1u, 2u * c->n_cu / nwin);  // one wave of 2 per CU
        }
      }
      if (sp_lists) {
        const uint64_t mean = budget / sp_nwin;
        g.sp_nwin = (uint32_t)sp_nwin;
        uint64_t cap = (mean + mean / 4 + 64 + 1) & ~1ULL;  // even: 16-byte key pairs
        if (!c->sv.compact)  // 32- (narrow: 24-) byte entries: wide_list_bytes of lists per ctx
          cap = std::max<uint64_t>(16, c->wide_list_bytes / (8 * list_words) / ((uint64_t)a.blocks * sp_nwin)) &
                ~1ULL;
        g.sp_cap = (uint32_t)cap;
      }
      return g;
    };
    auto geom_of = [](const LaunchArgs &x) {
      Geom g;
      if (x.spill) {
        g.nwin = x.nwin;
        g.spill_cap = x.spill_cap;
        g.win_blocks = x.win_blocks;
        g.win_shift = x.win_shift;
      }
      if (x.sp_lists) {
        g.sp_nwin = x.sp_nwin;
        g.sp_cap = x.sp_cap;
      }
      return g;
    };
    // Deferred folds: while the geometry holds, launches keep appending to the same lists
    // (their counters start from the stored fill) for up to kDeferLaunches (64) launches' worth
    // of records per workgroup, and fold_pending folds them once.
    // Plans with compact-key lists always defer: their fold pays a fixed pass over the
    // group-by table.  Spill-only plans (C2, C4) defer only small launches (at most
    // kMaxRecordsPerBlock / kDeferLaunches records per workgroup, e.g. the Go plugin's 2^20
    // records): there the spill fold's fixed pass over the windows cost more than the
    // tier-1 kernel itself; at full-size launches appending past earlier launches' entries
    // measured ~2 % slower in the tier-1 kernel (profiles/round2/r4f_*), so they fold per batch.
    const bool small_spill = c->dense_len > a.lds_bins && a.chunk <= kSmallLaunchChunk;
    const bool lists = sp_lists || small_spill;
    const bool defer = c->defer_folds && lists;
    // Wide lists (192-bit keys) are folded when the device says so: every launch's fold
    // skips itself until some list is half full (sparse_fold_wide_kernel), so the host keeps
    // appending without a record budget -- under skew the LDS hot-key cache absorbs most
    // updates and a budget that assumes one entry per record folded ~5x too often.
    const bool fold_cond = defer && sp_lists && !c->sv.compact;
    uint64_t budget = defer ? std::max<uint64_t>(a.chunk, std::min<uint64_t>(kMaxRecordsPerBlock,
                                                                             kDeferLaunches * a.chunk))
                            : a.chunk;
    if (fold_cond) budget = ~0ull >> 1;
    bool accum = false;
    if (c->pend.active) {
      const LaunchArgs &q = c->pend.a;
      const Geom pg = geom(c->pend.budget);
      accum = defer && c->pend.rpb + a.chunk <= c->pend.budget && pg == geom_of(q) && q.blocks == a.blocks &&
              q.lds_bins == a.lds_bins && q.dense_len == c->dense_len && q.dense_cnt == c->d_dense_cnt &&
              q.dense_byt == c->d_dense_byt && q.sparse.k0 == c->sv.k0;
      if (accum) budget = c->pend.budget;
      else if ((rc = fold_pending_dense(c))) return rc;
    }
    const Geom g = geom(budget);
    if (g.nwin) {
      if ((rc = ensure_buf(c, &c->d_spill, &c->spill_alloc, (size_t)a.blocks * g.nwin * g.spill_cap))) return rc;
      if ((rc = ensure_buf(c, &c->d_spill_count, &c->spill_count_alloc, (size_t)a.blocks * g.nwin))) return rc;
      a.spill_cap = g.spill_cap;
      a.spill = c->d_spill;
      a.spill_count = c->d_spill_count;
      a.nwin = g.nwin;
      a.spill_lo = a.lds_bins;
      a.win_shift = g.win_shift;
      a.win_blocks = g.win_blocks;
      // fold partials are stored (not atomically added) and summed by a reduce pass
      const size_t nb_stage = (size_t)a.win_blocks << a.win_shift;
      if ((rc = ensure_buf(c, &c->d_stage_b, &c->stage_b_alloc, nb_stage))) return rc;
      a.stage_b = c->d_stage_b;
    }
    a.sp_lists = nullptr;
    a.sp_counts = nullptr;
    a.sp_nwin = 0;
    if (g.sp_nwin) {
      if ((rc = ensure_buf(c, &c->d_sp_lists, &c->sp_lists_alloc,
                           (size_t)a.blocks * g.sp_nwin * g.sp_cap * list_words)))
        return rc;
      if ((rc = ensure_buf(c, &c->d_sp_counts, &c->sp_counts_alloc, (size_t)a.blocks * g.sp_nwin))) return rc;
      a.sp_lists = c->d_sp_lists;
      a.sp_counts = c->d_sp_counts;
      a.sp_nwin = g.sp_nwin;
      a.sp_cap = g.sp_cap;
    }
    a.accum = accum;
    a.defer_folds = defer && (a.spill || a.sp_lists);
    // small spill-only launches keep the tier-1 copies too: each workgroup continues from
    // its staged copy and the copies are summed once, by the deferred fold -- the per-launch
    // stage_reduce_kernel (reading blocks x the LDS bins) was most of such a launch's cost
    a.stage_defer = a.defer_folds && small_spill && !sp_lists && a.stage_a != nullptr;
    a.stage_accum = a.stage_defer && accum && c->pend.a.stage_defer && c->pend.a.stage_a == a.stage_a &&
                    c->pend.a.stage_a_stride == a.stage_a_stride;
    a.fold_cond = false;
    a.fold_flag = nullptr;
    if (fold_cond && a.sp_lists) {
      if (!c->d_fold_flag) {
        if ((rc = dev_alloc(c, &c->d_fold_flag, 2))) return rc;
        HIPCHK(c, x_set_async(c, c->d_fold_flag, 0, 8, c->stream));
      }
      a.fold_cond = true;
      a.fold_flag = c->d_fold_flag;
      a.fold_parity = c->fold_parity;
      c->fold_parity ^= 1u;
    }
    a.dense_cnt = c->d_dense_cnt;
    a.dense_byt = c->d_dense_byt;
    std::array<hipEvent_t, 3> ev{};
    if (c->timing) {
      if (c->tm_chain && c->tm_end) {
        ev[0] = c->tm_end;  // the previous launch's end: nothing ran in between
      } else {
        HIPCHK(c, hipEventCreateWithFlags(&ev[0], kTimingEventFlags));
        HIPCHK(c, hipEventRecord(ev[0], c->stream));
      }
      HIPCHK(c, hipEventCreateWithFlags(&ev[1], kTimingEventFlags));
      HIPCHK(c, hipEventCreateWithFlags(&ev[2], kTimingEventFlags));
    }
    const char *kname = nullptr;
    HIPCHK(c, launch_aggregate(a, c->stream, c->timing ? ev[1] : nullptr, &kname));
    if (kname) c->kernel_name = kname;
    if (a.defer_folds) {
      c->pend.rpb = (accum ? c->pend.rpb : 0) + a.chunk;
      c->pend.budget = budget;
      c->pend.a = a;
      c->pend.active = true;
    }
    if (c->timing) {
      HIPCHK(c, hipEventRecord(ev[2], c->stream));
      c->pending_events.push_back(ev);
      c->tm_end = ev[2];
      c->tm_chain = true;
    }
  }
  if ((c->cms_len || c->hll_len) && (rc = launch_sketches(c, cv, n))) return rc;
  if (c->lat_enabled && (rc = launch_latency(c, cv, n))) return rc;
  c->stats.records += n;
  c->stats.batches += 1;
  c->stats.last_kernel = a.tier1 ? GPUAGG_KERNEL_DENSE_LDS_IP
                         : a.dense_ng ? GPUAGG_KERNEL_DENSE_HBM_IP : GPUAGG_KERNEL_GENERIC;
  return GPUAGG_OK;
}

// Decodes n raw records at dev_raw into `out` on the ctx's stream (timed when enabled).
int decode(gpuagg_ctx *c, int kind, const void *dev_raw, size_t n, const OutCols &out) {
  if (kind != kRawPacket && kind != kRawDrop) return fail(c, GPUAGG_EINVAL, "unknown raw record kind %d", kind);
  if (n == 0) return GPUAGG_OK;
  if (!dev_raw || (!c->cpu && ((uintptr_t)dev_raw & 15u)))
    return fail(c, GPUAGG_EINVAL, "raw records must be 16-byte aligned");
  if (!out.src_ip || !out.dst_ip || !out.bytes || !out.meta) return fail(c, GPUAGG_EINVAL, "decode: null column");
  if (!c->d_decode_oor) {
    if (int rc = dev_alloc(c, &c->d_decode_oor, 1)) return rc;
    HIPCHK(c, x_set_async(c, c->d_decode_oor, 0, 8, c->stream));
  }
  if (c->cpu) {
    *c->d_decode_oor += c->cpu->decode(DecodeArgs{kind, dev_raw, n, out, c->d_decode_oor, c->n_cu,
                                                  (uint64_t)c->time_offset});
    c->stats.decoded += n;
    return GPUAGG_OK;
  }
  std::array<hipEvent_t, 2> ev{};
  if (c->timing) {
    for (auto &e : ev) HIPCHK(c, hipEventCreateWithFlags(&e, kTimingEventFlags));
    HIPCHK(c, hipEventRecord(ev[0], c->stream));
  }
  DecodeArgs a{kind, dev_raw, n, out, c->d_decode_oor, c->n_cu, (uint64_t)c->time_offset};
  ENQ(c);
  HIPCHK(c, launch_decode(a, c->stream));
  if (c->timing) {
    HIPCHK(c, hipEventRecord(ev[1], c->stream));
    c->pending_decode.push_back(ev);
  }
  c->stats.decoded += n;
  return GPUAGG_OK;
}

// Decodes into staging buffer s's columns and aggregates from there.
int decode_and_launch(gpuagg_ctx *c, gpuagg_ctx::Staging &s, int kind, const void *dev_raw, size_t n) {
  int rc;
  uint32_t *const *d = s.cols;
  const bool lat = c->lat_enabled != 0;
  const OutCols out{d[0], d[1], d[2], d[3], (c->plan.need_ports || c->cms_len > 0 || lat) ? d[4] : nullptr,
                    c->plan.need_dns ? d[5] : nullptr, lat ? s.tcp_id : nullptr, lat ? s.time_ns : nullptr};
  if ((rc = decode(c, kind, dev_raw, n, out))) return rc;
  ColsView cv{d[0], d[1], d[2], d[3], d[4], d[5], s.tcp_id, s.time_ns};
  return launch(c, cv, n);
}

}  // namespace

// ======================================================================================
extern "C" {

int gpuagg_create(const gpuagg_config *cfg, gpuagg_ctx **out) {
  if (!cfg || !out) return GPUAGG_EINVAL;
  *out = nullptr;
  if (cfg->abi_version != GPUAGG_ABI_VERSION) return GPUAGG_EINVAL;
  std::unique_ptr<gpuagg_ctx> c(new gpuagg_ctx());
  c->cfg = *cfg;
  c->device = cfg->device;
  c->remote = cfg->remote_context != 0;
  if (cfg->max_slots == 0 || cfg->max_slots > kMaxSlot + 1) return GPUAGG_EINVAL;
  if (cfg->cms_depth && (cfg->cms_width_log2 < 4 || cfg->cms_width_log2 > 28 || cfg->cms_depth > 16))
    return GPUAGG_EINVAL;
  if (cfg->hll_precision && (cfg->hll_precision < 4 || cfg->hll_precision > 18)) return GPUAGG_EINVAL;
  if (cfg->latency_limit > (1u << 26)) return GPUAGG_EINVAL;
  if (cfg->flags & GPUAGG_FLAG_CPU_BACKEND) {
    // host threads instead of a device: the node's CPU share (GPUAGG_CPU_THREADS, else the
    // hardware threads, at most 64)
    unsigned t = std::thread::hardware_concurrency();
    if (const char *e = getenv("GPUAGG_CPU_THREADS")) t = (unsigned)atoi(e);
    t = std::max(1u, std::min(64u, t ? t : 1u));
    c->cpu.reset(new cpu::Engine(t));
    c->cfg.flags |= GPUAGG_FLAG_NO_LDS_IP_TABLE;  // no LDS images to build
    c->n_cu = t;
    c->defer_folds = false;
    if (cfg->cms_depth) {
      c->cms_len = (size_t)cfg->cms_depth << cfg->cms_width_log2;
      if (dev_alloc(c.get(), &c->d_cms, c->cms_len)) return GPUAGG_ENOMEM;
    }
    *out = c.release();
    return GPUAGG_OK;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= c->device || c->device < 0)
    return GPUAGG_EDEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) return GPUAGG_EDEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return GPUAGG_EDEVICE;  // built for gfx950 only
  if (hipSetDevice(c->device) != hipSuccess) return GPUAGG_EDEVICE;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) {
    gpuagg_destroy(c.release());
    return GPUAGG_EDEVICE;
  }
  for (auto &st : c->stg)
    if (hipEventCreateWithFlags(&st.copied, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&st.released, hipEventDisableTiming) != hipSuccess) {
      gpuagg_destroy(c.release());
      return GPUAGG_EDEVICE;
    }
  if (hipEventCreateWithFlags(&c->enrich_done, hipEventDisableTiming) != hipSuccess) {
    gpuagg_destroy(c.release());
    return GPUAGG_EDEVICE;
  }
  c->n_cu = (uint32_t)prop.multiProcessorCount;
  c->wide_list_bytes = cfg->wide_list_mib ? (uint64_t)cfg->wide_list_mib << 20
                                          : std::min<uint64_t>(kWideListBytes, (uint64_t)prop.totalGlobalMem / 8);
  c->defer_folds = !(cfg->flags & GPUAGG_FLAG_FOLD_PER_BATCH);
  if (cfg->cms_depth) {
    c->cms_len = (size_t)cfg->cms_depth << cfg->cms_width_log2;
    if (dev_alloc(c.get(), &c->d_cms, c->cms_len)) {
      gpuagg_destroy(c.release());
      return GPUAGG_ENOMEM;
    }
  }
  if (layout_dense(c.get(), key_cap_for(c.get(), 0), false) || reset_state(c.get())) {
    gpuagg_destroy(c.release());
    return GPUAGG_EDEVICE;
  }
  *out = c.release();
  return GPUAGG_OK;
}

void gpuagg_destroy(gpuagg_ctx *c) {
  if (!c) return;
  if (!c->cpu) {
    hipSetDevice(c->device);
    if (c->copy_stream) hipStreamSynchronize(c->copy_stream);
    if (c->stream) hipStreamSynchronize(c->stream);
  }
  // feeds over this context release their stagings of it now and refuse further puts
  const std::vector<gpuagg_raw_feed *> feeds = c->feeds;
  for (gpuagg_raw_feed *f : feeds) gpuagg::feed_on_ctx_destroy(f, c);
  c->feeds.clear();
  drain_timing(c);
  for (auto *b : c->batches) {
    free_batch_cols(c, b);
    delete b;
  }
  dev_free(c, c->d_ip);
  dev_free(c, c->d_rpre);
  dev_free(c, c->d_rblk);
  dev_free(c, c->d_ipl);
  dev_free(c, c->d_ipl_all);
  dev_free(c, c->d_ipc);
  dev_free(c, c->d_api);
  dev_free(c, c->d_lat);
  dev_free(c, c->d_lat_blk_cnt);
  dev_free(c, c->d_lat_blk_max);
  dev_free(c, c->d_lat_blk_clk);
  dev_free(c, c->d_lat_blk_base);
  dev_free(c, c->d_lat_ev);
  dev_free(c, c->d_lat_hash);
  dev_free(c, c->d_lat_idx);
  dev_free(c, c->d_lat_delta);
  dev_free(c, c->d_lat_max_live);
  dev_free(c, c->d_lat_okeys);
  dev_free(c, c->d_lat_ovals);
  dev_free(c, c->d_lat_carry[0]);
  dev_free(c, c->d_lat_carry[1]);
  if (c->d_lat_tmp) hipFree(c->d_lat_tmp);
  x_host_free(c, c->h_lat_n);
  x_host_free(c, c->h_sync_words);
  dev_free(c, c->d_dense_cnt);
  dev_free(c, c->d_dense_byt);
  dev_free(c, c->sv.k0);  // k1, k2, cnt, byt point into the same array
  dev_free(c, c->sv.dropped);
  dev_free(c, c->d_counter);
  dev_free(c, c->d_export);
  dev_free(c, c->d_cms);
  dev_free(c, c->d_hll);
  dev_free(c, c->d_spill);
  dev_free(c, c->d_spill_count);
  dev_free(c, c->d_stage_a);
  dev_free(c, c->d_fold_flag);
  dev_free(c, c->d_enrich);
  dev_free(c, c->d_stage_b);
  dev_free(c, c->d_sk_lists);
  dev_free(c, c->d_sk_counts);
  dev_free(c, c->d_sp_lists);
  dev_free(c, c->d_sp_counts);
  dev_free(c, c->d_hll_lists);
  dev_free(c, c->d_hll_lists2);
  dev_free(c, c->d_hll_counts2);
  dev_free(c, c->d_hll_counts);
  dev_free(c, c->d_decode_oor);
  for (auto &st : c->stg) {
    for (auto &p : st.cols) dev_free(c, p);
    dev_free(c, st.raw);
    if (st.copied) hipEventDestroy(st.copied);
    if (st.released) hipEventDestroy(st.released);
  }
  if (c->enrich_done) {
    hipEventDestroy(c->enrich_done);
  }
  for (ncclComm_t cm : c->rccl_comms) ncclCommDestroy(cm);
  c->rccl_comms.clear();
  if (c->fold_stream) {
    hipStreamSynchronize(c->fold_stream);
    hipStreamDestroy(c->fold_stream);
  }
  if (c->fold_fork) hipEventDestroy(c->fold_fork);
  if (c->fold_join) hipEventDestroy(c->fold_join);
  if (c->copy_stream) hipStreamDestroy(c->copy_stream);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

const char *gpuagg_last_error(const gpuagg_ctx *c) { return c ? c->err.c_str() : "null ctx"; }

// validations.MetricsContextOptionsCompare (validate_metricconfiguration.go:118-160):
// same number of entries, same metric names (last entry of a name wins), source and
// destination label lists equal as sets (utils.CompareStringSlice, common.go:58-84).
bool same_options(const std::vector<OptCopy> &a, const std::vector<OptCopy> &b) {
  if (a.size() != b.size()) return false;
  std::map<std::string, const OptCopy *> ma, mb;
  for (auto &o : a) ma[o.name] = &o;
  for (auto &o : b) mb[o.name] = &o;
  if (ma.size() != mb.size()) return false;
  auto same_set = [](const std::vector<std::string> &x, const std::vector<std::string> &y) {
    if (x.size() != y.size()) return false;
    std::set<std::string> sx(x.begin(), x.end()), sy(y.begin(), y.end());
    return sx == sy;
  };
  for (auto &kv : ma) {
    auto it = mb.find(kv.first);
    if (it == mb.end()) return false;
    if (!same_set(kv.second->src, it->second->src) || !same_set(kv.second->dst, it->second->dst)) return false;
  }
  return true;
}

int gpuagg_reconcile(gpuagg_ctx *c, const gpuagg_metric_options *opts, size_t n) {
  if (!c || (n && !opts)) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  std::vector<OptCopy> new_opts(n);
  for (size_t i = 0; i < n; ++i) {
    new_opts[i].name = opts[i].metric_name ? opts[i].metric_name : "";
    for (uint32_t k = 0; opts[i].source_labels && k < opts[i].n_source_labels; ++k)
      new_opts[i].src.push_back(opts[i].source_labels[k] ? opts[i].source_labels[k] : "");
    for (uint32_t k = 0; opts[i].destination_labels && k < opts[i].n_destination_labels; ++k)
      new_opts[i].dst.push_back(opts[i].destination_labels[k] ? opts[i].destination_labels[k] : "");
  }
  // Module.Reconcile leaves the metrics alone when the context options compare equal
  // (metrics_module.go:142-166): a resync or a namespace-only change keeps the counters
  if (c->have_opts && same_options(c->cur_opts, new_opts)) return GPUAGG_OK;
  HIPCHK(c, x_sync(c, c->stream));
  const bool local = !c->remote;
  // NewLatencyMetrics (latency.go:73-115): the three names it switches on
  uint32_t lat = 0;
  for (const auto &o : new_opts) {
    if (o.name == "node_apiserver_latency") lat |= 1u;
    else if (o.name == "node_apiserver_handshake_latency") lat |= 2u;
    else if (o.name == "node_apiserver_no_response") lat |= 4u;
  }

  // Module.updateMetricsContexts: registry keyed by MetricName, last writer wins.
  std::map<std::string, Instance> registry;
  for (size_t i = 0; i < n; ++i) {
    const gpuagg_metric_options &o = opts[i];
    const std::string name = o.metric_name ? o.metric_name : "";
    const std::string lname = lower(name.c_str());
    Instance in{};
    in.registry_name = name;
    in.has_src = local ? o.source_labels_set != 0 : o.source_labels_set != 0;
    in.has_dst = local ? false : o.destination_labels_set != 0;
    in.src_opts = in.has_src ? parse_opts(o.source_labels, o.n_source_labels) : 0;
    in.dst_opts = in.has_dst ? parse_opts(o.destination_labels, o.n_destination_labels) : 0;
    in.adv_enable = name != "" && (o.n_source_labels > 0 || o.n_destination_labels > 0);
    bool make = false;
    if (name.find("forward") != std::string::npos) {
      make = lname.find("forward") != std::string::npos;
      in.family = FAM_FWD;
      in.active = name == "forward_count" || name == "forward_bytes";
      in.vk = name == "forward_bytes" ? VK_BYTES : VK_COUNT;
      in.vec_name = name == "forward_bytes" ? "adv_forward_bytes" : "adv_forward_count";
    } else if (name.find("drop") != std::string::npos) {
      make = true;
      in.family = FAM_DROP;
      in.active = name == "drop_count" || name == "drop_bytes";
      in.vk = name == "drop_bytes" ? VK_BYTES : VK_COUNT;
      in.vec_name = name == "drop_bytes" ? "adv_drop_bytes" : "adv_drop_count";
    } else if (name.find("tcp") != std::string::npos) {
      if (lname.find("retrans") != std::string::npos) {  // NewTCPRetransMetrics overwrites
        make = true;
        in.family = FAM_RETRANS;
        in.vec_name = "adv_tcpretrans_count";
        in.active = true;
      } else if (lname.find("flag") != std::string::npos) {
        make = true;
        in.family = FAM_TCPFLAGS;
        in.vec_name = "adv_tcpflags_count";
        in.active = true;
      }
      in.vk = VK_COUNT;
    } else if (name.find("node_apiserver") != std::string::npos) {
      make = false;  // latency metrics: next, not part of this path yet
    } else if (name.find("dns") != std::string::npos || name.find("pktmon") != std::string::npos) {
      if (lname.find("dns") != std::string::npos) {
        make = true;
        in.vk = VK_COUNT;
        if (name == "dns_request_count") {
          in.family = FAM_DNS_REQ;
          in.vec_name = "adv_dns_request_count";
        } else if (name == "dns_response_count") {
          in.family = FAM_DNS_RESP;
          in.vec_name = "adv_dns_response_count";
        } else {
          return fail(c, GPUAGG_EINVAL,
                      "metric %s: DNS metric with no vector (dns.go:352-372 leaves it nil and the "
                      "first DNS flow would panic)", name.c_str());
        }
        in.active = true;
      }
    }
    if (!make) continue;
    if (local && in.active && !in.has_src)
      return fail(c, GPUAGG_EINVAL,
                  "metric %s: local context needs sourceLabels (srcCtx is nil, basemetricsobject.go:32-39)",
                  name.c_str());
    registry[name] = in;
  }

  // label schemas
  std::map<std::string, int> fam_seen;
  std::vector<Instance> inst;
  for (auto &kv : registry) {
    Instance in = kv.second;
    std::vector<std::string> ln;
    switch (in.family) {
      case FAM_FWD: ln = {"direction"}; break;
      case FAM_DROP: ln = {"reason", "direction"}; break;
      case FAM_TCPFLAGS: ln = {"flag"}; break;
      case FAM_RETRANS: ln = {"direction"}; break;
      case FAM_DNS_REQ: ln = {"query_type", "query"}; break;
      case FAM_DNS_RESP: ln = {"return_code", "query_type", "query", "response", "num_response"}; break;
    }
    const bool ctx_labels = in.family != FAM_FWD || in.adv_enable;
    if (ctx_labels) {
      if (local) {
        if (in.has_src) ctx_label_names(in.src_opts, "", ln);
      } else {
        if (in.has_src) ctx_label_names(in.src_opts, "source_", ln);
        if (in.has_dst) ctx_label_names(in.dst_opts, "destination_", ln);
      }
    }
    in.label_names = ln;
    in.vec_name = std::string("networkobservability_") + in.vec_name;
    if (in.active) {
      if (fam_seen.count(in.vec_name))
        return fail(c, GPUAGG_EDUPLICATE, "metrics %s and %s both register %s",
                    registry.count(in.registry_name) ? in.registry_name.c_str() : "?",
                    inst[fam_seen[in.vec_name]].registry_name.c_str(), in.vec_name.c_str());
      fam_seen[in.vec_name] = (int)inst.size();
    }
    inst.push_back(in);
  }

  // groups: one per (family, effective options)
  std::vector<Group> groups;
  for (auto &in : inst) {
    in.group = -1;
    if (!in.active) continue;
    uint8_t so = in.has_src ? in.src_opts : 0, dopt = in.has_dst ? in.dst_opts : 0;
    if (in.family == FAM_FWD && !in.adv_enable) so = dopt = 0;
    if (local && so == 0) continue;  // getLocalCtxValues yields no values: no updates
    int gi = -1;
    for (size_t g = 0; g < groups.size(); ++g)
      if (groups[g].family == in.family && groups[g].src_opts == so && groups[g].dst_opts == dopt) gi = (int)g;
    if (gi < 0) {
      if (groups.size() >= (size_t)kMaxGroups)
        return fail(c, GPUAGG_ECAPACITY, "more than %d metric groups", kMaxGroups);
      Group g{};
      g.family = in.family;
      g.src_opts = so;
      g.dst_opts = dopt;
      const bool dns = in.family == FAM_DNS_REQ || in.family == FAM_DNS_RESP;
      g.sparse = !local || dns || (so & (OPT_IP | OPT_PORT));
      if (!g.sparse) {
        g.key_mode = (so & OPT_EP) ? 1 : 0;
        g.nkeys = 0;  // laid out by layout_dense
        g.nsub = (in.family == FAM_DROP || in.family == FAM_TCPFLAGS) ? 8 : 1;
      }
      groups.push_back(g);
      gi = (int)groups.size() - 1;
    }
    in.group = gi;
  }

  // Dense bin layout, hottest family first: bins [0, L) live in LDS (kernels file), so
  // forward counters (every forwarded flow) go before TCP-flag, drop and retransmit ones.
  {
    // Group indices follow the same order (dense groups in layout order, then sparse
    // ones), so the tier-1 kernel's compile-time signatures see group 0 = hottest.
    static const int prio[FAM_COUNT] = {0, 2, 1, 3, 9, 9};
    std::vector<size_t> order(groups.size());
    for (size_t g = 0; g < groups.size(); ++g) order[g] = g;
    std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {
      if (groups[x].sparse != groups[y].sparse) return !groups[x].sparse;
      return !groups[x].sparse && prio[groups[x].family] < prio[groups[y].family];
    });
    std::vector<Group> sorted;
    std::vector<int> new_index(groups.size());
    for (size_t i = 0; i < order.size(); ++i) {
      new_index[order[i]] = (int)i;
      sorted.push_back(groups[order[i]]);
    }
    groups.swap(sorted);
    for (auto &in : inst)
      if (in.group >= 0) in.group = new_index[in.group];
  }

  Plan p{};
  p.local = local ? 1 : 0;
  p.ngroups = (int32_t)groups.size();
  bool any_sparse = false;
  for (size_t g = 0; g < groups.size(); ++g) {
    GroupPlan &gp = p.g[g];
    gp.family = groups[g].family;
    gp.sparse = groups[g].sparse;
    gp.src_opts = groups[g].src_opts;
    gp.dst_opts = groups[g].dst_opts;
    gp.nsub = groups[g].nsub;
    gp.key_mode = groups[g].key_mode;
    if ((gp.src_opts | gp.dst_opts) & OPT_PORT) p.need_ports = 1;
    if (gp.family == FAM_DNS_REQ || gp.family == FAM_DNS_RESP) p.need_dns = 1;
    if (gp.family == FAM_FWD || gp.family == FAM_DROP) p.need_bytes = 1;
    any_sparse |= groups[g].sparse;
  }

  // (re)allocate state: dense counters for the slots in use, zeroed
  if (any_sparse && (rc = ensure_sparse(c))) return rc;
  // compact group-by keys when every sparse key fits 64 bits: local context whose only
  // sparse groups are DNS without ip / port options (key = group|side|slot|dns id)
  bool compact = local && any_sparse;
  for (size_t g = 0; g < groups.size(); ++g)
    if (groups[g].sparse)
      compact &= (groups[g].family == FAM_DNS_REQ || groups[g].family == FAM_DNS_RESP) &&
                 !(groups[g].src_opts & (OPT_IP | OPT_PORT));
  c->sv.compact = compact ? 1u : 0u;
  // wide keys with no port / DNS fields may take 24-byte list entries (kWideNarrowWords) on
  // request: fewer bytes, but written as partial sectors
  c->sv.narrow = (!compact && !p.need_ports && !p.need_dns && (c->cfg.flags & GPUAGG_FLAG_NARROW_ENTRIES)) ? 1u : 0u;
  if (c->sparse_slots) {  // probe / fold segments: compact 2^13 slots; wide 2^12 (or the table)
    const uint32_t lg = (uint32_t)__builtin_ctzll(c->sparse_slots);
    c->sv.seg_log2 = compact ? std::min<uint32_t>(lg, kSparseSegLog2)
                             : (lg <= kWideMaxLog2 ? std::min<uint32_t>(lg, kWideSegLog2) : lg);
  }
  c->inst = inst;
  c->groups = groups;
  c->plan = p;
  if ((rc = layout_dense(c, key_cap_for(c, c->slots.size()), false))) return rc;
  c->cur_opts = new_opts;
  c->have_opts = true;
  c->lat_enabled = lat;
  if ((rc = lat_reset(c, true))) return rc;  // Init: a new TTL cache (latency.go:118-122)
  return reset_state(c);
}

int gpuagg_slot_intern(gpuagg_ctx *c, const char *ns, const char *pod, const char *wk_kind,
                       const char *wk_name, int32_t *slot) {
  if (!c || !ns || !pod || !slot) return GPUAGG_EINVAL;
  const int has_owner = wk_kind != nullptr;
  auto key = std::make_tuple(std::string(ns), std::string(pod), std::string(has_owner ? wk_kind : ""),
                             std::string(has_owner && wk_name ? wk_name : ""), has_owner);
  auto it = c->slot_ids.find(key);
  if (it != c->slot_ids.end()) {
    *slot = it->second;
    return GPUAGG_OK;
  }
  if (c->free_slots.empty() && c->slots.size() >= c->cfg.max_slots)
    return fail(c, GPUAGG_ECAPACITY, "more than max_slots=%u endpoint identities (retire unused ones "
                "with gpuagg_retire_slots)", c->cfg.max_slots);
  SlotAttr a;
  a.ns = ns;
  a.pod = pod;
  a.has_owner = has_owner;
  if (has_owner) {
    a.wk_kind = wk_kind;
    a.wk_name = wk_name ? wk_name : "";
  }
  a.api = a.ns == kApiServer && a.pod == kApiServer;
  int32_t id;
  if (!c->free_slots.empty()) {  // a retired id: its state was cleared when it retired
    id = c->free_slots.back();
    c->free_slots.pop_back();
    c->slots[id] = a;
  } else {
    id = (int32_t)c->slots.size();
    c->slots.push_back(a);
  }
  ++c->slots_version;
  c->slot_ids.emplace(key, id);
  *slot = id;
  return GPUAGG_OK;
}

// An LDS image of (ip, slot) entries in the cheapest form the set allows: dense radix
// (one u16 read per lookup), radix with its row table (two), else the bucketized cuckoo
// table.  GPUAGG_FLAG_LDS_CUCKOO / GPUAGG_FLAG_ROW_RADIX force the latter forms
// (diagnostics and tests).
struct LdsImage {
  bool radix = false, dense = false;
  uint32_t nb = 0, seed = 0, npfx = 0;
  uint32_t pfx[kIprMaxPfx] = {kIprNoPfx, kIprNoPfx, kIprNoPfx, kIprNoPfx}, dr[kIprMaxPfx] = {};
  std::vector<uint8_t> bytes;
};
bool build_lds_image(const std::vector<std::pair<uint32_t, uint32_t>> &ents, uint32_t flags, LdsImage *out) {
  if (!(flags & GPUAGG_FLAG_LDS_CUCKOO)) {
    IprdImage id;
    if (!(flags & GPUAGG_FLAG_ROW_RADIX) && iprd_build(ents, &id)) {
      out->radix = out->dense = true;
      out->npfx = id.npfx;
      for (uint32_t j = 0; j < kIprMaxPfx; ++j) {
        out->pfx[j] = id.pfx[j];
        out->dr[j] = id.dr[j];
      }
      out->bytes = std::move(id.bytes);
      return true;
    }
    IprImage ir;
    if (ipr_build(ents, &ir)) {
      out->radix = true;
      out->npfx = ir.npfx;
      for (uint32_t j = 0; j < kIprMaxPfx; ++j) out->pfx[j] = ir.pfx[j];
      out->bytes = std::move(ir.bytes);
      return true;
    }
  }
  IplImage im;
  if (!ipl_build(ents, &im)) return false;
  out->nb = im.nb;
  out->seed = im.seed;
  out->bytes = std::move(im.bytes);
  return true;
}

int gpuagg_set_endpoints(gpuagg_ctx *c, const uint32_t *ipv4, const int32_t *slot, size_t n,
                         uint64_t version) {
  if (!c || (n && (!ipv4 || !slot))) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  if (n > c->cfg.max_ips) return fail(c, GPUAGG_ECAPACITY, "%zu IPs exceed max_ips=%u", n, c->cfg.max_ips);
  // last writer wins for an IP held twice (cache.go:204-233)
  std::unordered_map<uint32_t, uint64_t> last;
  last.reserve(n * 2 + 1);
  for (size_t i = 0; i < n; ++i) {
    if (slot[i] < 0 || (size_t)slot[i] >= c->slots.size() || !c->slots[slot[i]].in_use)
      return fail(c, GPUAGG_EINVAL, "entry %zu: slot %d was not interned", i, slot[i]);
    if (ipv4[i] == 0xFFFFFFFFu) return fail(c, GPUAGG_ERANGE, "255.255.255.255 cannot be a pod IP");
    last[ipv4[i]] = ip_entry(ipv4[i], (uint32_t)slot[i], c->slots[slot[i]].api);
  }
  // Bucketized cuckoo build: buckets of 2 entries (16 bytes, one load), two choices,
  // first choice preferred; an entry moves to its second bucket only while its first is
  // full, and a kick always refills the bucket it empties, so "key in its second bucket
  // => first bucket full" holds and a lookup stops after the first bucket whenever that
  // bucket has a free slot.  Load <= 40 %; re-seed on a failed insertion, grow after 8.
  size_t cap = 64;  // entries (2 per bucket)
  while (cap * 40 < last.size() * 100) cap <<= 1;
  std::vector<uint64_t> tab;
  uint32_t seed = 0x2545F491u;
  for (int attempt = 0;; ++attempt) {
    if (attempt && attempt % 8 == 0) cap <<= 1;
    seed = (uint32_t)fmix64((uint64_t)seed + 0x9E3779B97F4A7C15ULL * (attempt + 1));
    tab.assign(cap, kIpEmpty);
    const uint32_t bmask = (uint32_t)(cap / 2 - 1);
    uint64_t rnd = 0x9E3779B97F4A7C15ULL ^ seed;
    auto put = [&](uint32_t b, uint64_t e) {
      for (int k = 0; k < 2; ++k)
        if (tab[2 * b + k] == kIpEmpty) {
          tab[2 * b + k] = e;
          return true;
        }
      return false;
    };
    bool ok = true;
    for (const auto &kv : last) {
      uint64_t cur = kv.second;
      const uint32_t b1 = ip_h1((uint32_t)cur, seed) & bmask, b2 = ip_h2((uint32_t)cur, seed) & bmask;
      if (put(b1, cur) || put(b2, cur)) continue;
      uint32_t b = b2;  // both full: kick a random entry of the second bucket
      int kicks = 0;
      for (;;) {
        rnd = rnd * 6364136223846793005ULL + 1442695040888963407ULL;
        std::swap(cur, tab[2 * b + ((rnd >> 33) & 1)]);
        const uint32_t c1 = ip_h1((uint32_t)cur, seed) & bmask, c2 = ip_h2((uint32_t)cur, seed) & bmask;
        b = (b == c1) ? c2 : c1;  // the evicted key's other bucket
        if (put(b, cur)) break;
        if (++kicks > 500) {
          ok = false;
          break;
        }
      }
      if (!ok) break;
    }
    if (ok) break;
    if (cap > ((size_t)1 << 30)) return fail(c, GPUAGG_ECAPACITY, "IP table cannot be built");
  }
  HIPCHK(c, x_sync(c, c->stream));  // in-flight batches use the old table
  // dense counters / HLL rows cover every interned slot
  if (c->slots.size() > c->key_cap && (rc = layout_dense(c, key_cap_for(c, c->slots.size()), true)))
    return rc;
  if (cap != c->ip_cap) {
    dev_free(c, c->d_ip);
    c->ip_cap = 0;
    if ((rc = dev_alloc(c, &c->d_ip, cap))) return rc;
  }
  HIPCHK(c, x_copy(c, c->d_ip, tab.data(), cap * 8, hipMemcpyHostToDevice));
  c->ip_cap = cap;
  // radix image when the IPs fall in at most kRadixMaxBlocks /16 prefixes (cluster pod
  // CIDRs): L2-resident where a hash table of 100k+ IPs is not
  {
    std::map<uint32_t, uint32_t> blocks;  // prefix (low 16 bits of the LE u32) -> block
    for (const auto &kv : last) blocks.emplace(kv.first & 0xFFFFu, 0u);
    c->radix = !(c->cfg.flags & GPUAGG_FLAG_NO_RADIX_IP_TABLE) && !blocks.empty() &&
               blocks.size() <= kRadixMaxBlocks;
    if (c->radix) {
      uint32_t nb = 0;
      for (auto &kv : blocks) kv.second = nb++;
      c->radix_n = nb;
      for (auto &p : c->radix_pfx) p = 0;
      for (auto &kv : blocks)
        if (kv.second < kRadixSmall) c->radix_pfx[kv.second / 2] |= kv.first << (16 * (kv.second & 1));
      std::vector<uint16_t> pre(1u << 16, (uint16_t)kRadixNoBlock);
      for (auto &kv : blocks) pre[kv.first] = (uint16_t)kv.second;
      std::vector<uint32_t> blk((size_t)nb << 16, kRadixEmpty);
      for (const auto &kv : last) {
        const uint32_t sl = (uint32_t)((kv.second >> 32) & ((1u << kSlotBits) - 1));
        const uint32_t api = (uint32_t)(kv.second >> 53) & 1u;
        blk[((size_t)blocks[kv.first & 0xFFFFu] << 16) | (kv.first >> 16)] = sl | (api << 31);
      }
      if (!c->d_rpre && (rc = dev_alloc(c, &c->d_rpre, (size_t)1 << 16))) return rc;
      if ((rc = ensure_buf(c, &c->d_rblk, &c->rblk_alloc, blk.size()))) return rc;
      HIPCHK(c, x_copy(c, c->d_rpre, pre.data(), pre.size() * 2, hipMemcpyHostToDevice));
      HIPCHK(c, x_copy(c, c->d_rblk, blk.data(), blk.size() * 4, hipMemcpyHostToDevice));
    }
  }
  // LDS image: non-apiserver pods only (local context treats the apiserver pseudo pod
  // like no endpoint), u16 slot ids
  c->ipl_bytes = 0;
  if (!(c->cfg.flags & GPUAGG_FLAG_NO_LDS_IP_TABLE)) {
    std::vector<std::pair<uint32_t, uint32_t>> ents;
    for (const auto &kv : last)
      if (!((kv.second >> 53) & 1))
        ents.emplace_back(kv.first, (uint32_t)((kv.second >> 32) & ((1u << kSlotBits) - 1)));
    LdsImage im;
    if (build_lds_image(ents, c->cfg.flags, &im)) {
      const uint32_t bytes = (uint32_t)im.bytes.size();
      if (bytes > c->ipl_alloc) {
        dev_free(c, c->d_ipl);
        c->ipl_alloc = 0;
        if ((rc = dev_alloc(c, &c->d_ipl, bytes))) return rc;
        c->ipl_alloc = bytes;
      }
      HIPCHK(c, x_copy(c, c->d_ipl, im.bytes.data(), bytes, hipMemcpyHostToDevice));
      c->ipl_radix = im.radix;
      c->ipl_dense = im.dense;
      c->ipl_nb = im.nb;
      c->ipl_seed = im.seed;
      c->ipl_npfx = im.npfx;
      for (uint32_t j = 0; j < kIprMaxPfx; ++j) {
        c->ipl_pfx[j] = im.pfx[j];
        c->ipl_dr[j] = im.dr[j];
      }
      c->ipl_bytes = bytes;
    }
  }
  // LDS image of every pod IP (the apiserver pseudo pod included: it is a source pod for
  // the HLL) for the sketch pass and the remote context's wide_kernel
  c->ipl_all_bytes = 0;
  if ((c->cfg.hll_precision || c->remote) && !(c->cfg.flags & GPUAGG_FLAG_NO_LDS_IP_TABLE)) {
    std::vector<std::pair<uint32_t, uint32_t>> ents;
    for (const auto &kv : last) ents.emplace_back(kv.first, (uint32_t)((kv.second >> 32) & ((1u << kSlotBits) - 1)));
    LdsImage im;
    if (build_lds_image(ents, c->cfg.flags, &im)) {
      const uint32_t bytes = (uint32_t)im.bytes.size();
      if (bytes > c->ipl_all_alloc) {
        dev_free(c, c->d_ipl_all);
        c->ipl_all_alloc = 0;
        if ((rc = dev_alloc(c, &c->d_ipl_all, bytes))) return rc;
        c->ipl_all_alloc = bytes;
      }
      HIPCHK(c, x_copy(c, c->d_ipl_all, im.bytes.data(), bytes, hipMemcpyHostToDevice));
      c->ipl_all_radix = im.radix;
      c->ipl_all_dense = im.dense;
      c->ipl_all_nb = im.nb;
      c->ipl_all_seed = im.seed;
      c->ipl_all_npfx = im.npfx;
      for (uint32_t j = 0; j < kIprMaxPfx; ++j) {
        c->ipl_all_pfx[j] = im.pfx[j];
        c->ipl_all_dr[j] = im.dr[j];
      }
      c->ipl_all_bytes = bytes;
    }
  }
  c->ip_seed = seed;
  c->ip_version = version;
  c->installed.clear();
  for (const auto &kv : last) c->installed.emplace_back(kv.first, (int32_t)((kv.second >> 32) & ((1u << kSlotBits) - 1)));
  return GPUAGG_OK;
}

// ---- the IP cache (cache.go), restated natively --------------------------------------
namespace {

int cache_delete_endpoint_key(gpuagg_ctx *c, const std::string &key) {  // deleteEndpoint (:315-337)
  auto it = c->ep_map.find(key);
  if (it == c->ep_map.end()) return GPUAGG_OK;  // "ignore the error if the endpoint is not found"
  for (uint32_t ip : it->second.ips) c->ip_to_ep.erase(ip);
  c->ep_map.erase(it);
  return GPUAGG_OK;
}
int cache_delete_svc_key(gpuagg_ctx *c, const std::string &key) {  // deleteSvc (:348-368)
  auto it = c->svc_map.find(key);
  if (it == c->svc_map.end()) return fail(c, GPUAGG_ENOTFOUND, "service not found in cache: %s", key.c_str());
  c->ip_to_svc.erase(it->second);
  c->svc_map.erase(it);
  return GPUAGG_OK;
}
int cache_delete_node_key(gpuagg_ctx *c, const std::string &name) {  // deleteNode (:379-392)
  auto it = c->node_map.find(name);
  if (it == c->node_map.end()) return fail(c, GPUAGG_ENOTFOUND, "node not found in cache: %s", name.c_str());
  c->ip_to_node.erase(it->second);
  c->node_map.erase(it);
  return GPUAGG_OK;
}
// deleteByIP (:394-420): the object holding ip, unless it is `key` itself; services first,
// then pods, then nodes
int cache_delete_by_ip(gpuagg_ctx *c, uint32_t ip, const std::string &key) {
  auto s = c->ip_to_svc.find(ip);
  if (s != c->ip_to_svc.end()) return s->second == key ? GPUAGG_OK : cache_delete_svc_key(c, std::string(s->second));
  auto e = c->ip_to_ep.find(ip);
  if (e != c->ip_to_ep.end()) return e->second == key ? GPUAGG_OK : cache_delete_endpoint_key(c, std::string(e->second));
  auto n = c->ip_to_node.find(ip);
  if (n != c->ip_to_node.end()) return n->second == key ? GPUAGG_OK : cache_delete_node_key(c, std::string(n->second));
  return GPUAGG_OK;
}
std::string ep_key(const char *ns, const char *name) { return std::string(ns) + "/" + name; }

}  // namespace

int gpuagg_cache_update_endpoint(gpuagg_ctx *c, const char *ns, const char *pod, const char *wk_kind,
                                 const char *wk_name, const uint32_t *ipv4, size_t n_ips) {
  if (!c || !ns || !pod || (n_ips && !ipv4)) return GPUAGG_EINVAL;
  const std::string key = ep_key(ns, pod);
  if (!n_ips) return fail(c, GPUAGG_EINVAL, "no IP found for endpoint %s", key.c_str());  // ep.IPs() error
  int32_t slot;
  int rc = gpuagg_slot_intern(c, ns, pod, wk_kind, wk_name, &slot);
  if (rc) return rc;
  for (size_t i = 0; i < n_ips; ++i)  // updateEndpoint (:204-233)
    if ((rc = cache_delete_by_ip(c, ipv4[i], key))) return rc;
  gpuagg_ctx::CacheEp &e = c->ep_map[key];
  e.slot = slot;
  e.ips.assign(ipv4, ipv4 + n_ips);
  for (size_t i = 0; i < n_ips; ++i) c->ip_to_ep[ipv4[i]] = key;
  return GPUAGG_OK;
}

int gpuagg_cache_delete_endpoint(gpuagg_ctx *c, const char *ns, const char *pod) {
  if (!c || !ns || !pod) return GPUAGG_EINVAL;
  return cache_delete_endpoint_key(c, ep_key(ns, pod));
}

int gpuagg_cache_update_service(gpuagg_ctx *c, const char *ns, const char *name, uint32_t ipv4) {
  if (!c || !ns || !name) return GPUAGG_EINVAL;
  const std::string key = ep_key(ns, name);
  int rc = cache_delete_by_ip(c, ipv4, key);  // updateSvc (:244-270)
  if (rc) return rc;
  c->ip_to_svc[ipv4] = key;
  c->svc_map[key] = ipv4;
  return GPUAGG_OK;
}

int gpuagg_cache_delete_service(gpuagg_ctx *c, const char *ns, const char *name) {
  if (!c || !ns || !name) return GPUAGG_EINVAL;
  return cache_delete_svc_key(c, ep_key(ns, name));
}

int gpuagg_cache_update_node(gpuagg_ctx *c, const char *name, uint32_t ipv4) {
  if (!c || !name) return GPUAGG_EINVAL;
  int rc = cache_delete_by_ip(c, ipv4, name);  // updateNode (:282-305)
  if (rc) return rc;
  c->node_map[name] = ipv4;
  c->ip_to_node[ipv4] = name;
  return GPUAGG_OK;
}

int gpuagg_cache_delete_node(gpuagg_ctx *c, const char *name) {
  if (!c || !name) return GPUAGG_EINVAL;
  return cache_delete_node_key(c, name);
}

int gpuagg_cache_commit(gpuagg_ctx *c, uint64_t version) {
  if (!c) return GPUAGG_EINVAL;
  // GetObjByIP (cache.go:154-169): an IP resolves to a pod when ipToEpKey names an
  // endpoint still in epMap (an IP an updated pod no longer lists keeps pointing at it)
  std::vector<uint32_t> ips;
  std::vector<int32_t> slots;
  ips.reserve(c->ip_to_ep.size());
  slots.reserve(c->ip_to_ep.size());
  for (const auto &kv : c->ip_to_ep) {
    auto e = c->ep_map.find(kv.second);
    if (e == c->ep_map.end()) continue;
    ips.push_back(kv.first);
    slots.push_back(e->second.slot);
  }
  return gpuagg_set_endpoints(c, ips.data(), slots.data(), ips.size(), version);
}

int gpuagg_retire_slots(gpuagg_ctx *c, size_t *n_retired) {
  if (!c) return GPUAGG_EINVAL;
  if (n_retired) *n_retired = 0;
  int rc = bind(c);
  if (rc) return rc;
  if ((rc = fold_pending(c))) return rc;
  HIPCHK(c, x_sync(c, c->stream));
  std::vector<char> live(c->slots.size(), 0);
  for (const auto &e : c->installed) live[e.second] = 1;
  std::vector<uint32_t> dead;
  for (size_t s = 0; s < c->slots.size(); ++s)
    if (c->slots[s].in_use && !live[s]) dead.push_back((uint32_t)s);
  if (dead.empty()) return GPUAGG_OK;
  // dense bins and HLL rows of the dead slots (slots < key_cap: set_endpoints grew it)
  std::vector<uint32_t> dead_dev;
  for (uint32_t s : dead)
    if (s < c->key_cap) dead_dev.push_back(s);
  if (!dead_dev.empty() && (c->dense_len || c->hll_len)) {
    uint32_t *d = nullptr;
    if ((rc = dev_alloc(c, &d, dead_dev.size()))) return rc;
    hipError_t e = x_copy_async(c, d, dead_dev.data(), dead_dev.size() * 4, hipMemcpyHostToDevice, c->stream);
    if (c->cpu) {
      if (e == hipSuccess)
        cpu::zero_slots(c->dense_len ? c->d_dense_cnt : nullptr, c->d_dense_byt, c->hll_len ? c->d_hll : nullptr,
                        c->cfg.hll_precision, d, (uint32_t)dead_dev.size(), c->plan);
    } else if (e == hipSuccess) {
      ENQ(c);
      e = launch_zero_slots(c->dense_len ? c->d_dense_cnt : nullptr, c->d_dense_byt, c->hll_len ? c->d_hll : nullptr,
                            c->cfg.hll_precision, d, (uint32_t)dead_dev.size(), c->plan, c->stream);
    }
    if (e == hipSuccess) e = x_sync(c, c->stream);
    dev_free(c, d);
    if (e != hipSuccess) return fail(c, GPUAGG_EDEVICE, "retire: %s", hipGetErrorString(e));
  }
  // group-by entries keyed by a dead slot (as source or destination): the table is
  // rebuilt without them (export, filter on the host, re-insert)
  if (c->sparse_slots) {
    std::vector<char> is_dead(c->slots.size() + 1, 0);  // indexed by slot + 1
    for (uint32_t s : dead) is_dead[s + 1] = 1;
    if (c->export_cap < c->sparse_slots) {
      dev_free(c, c->d_export);
      c->export_cap = 0;
      if ((rc = dev_alloc(c, &c->d_export, c->sparse_slots * kSparseEntryWords))) return rc;
      c->export_cap = c->sparse_slots;
    }
    size_t nent = 0;
    if ((rc = gpuagg_sparse_export(c, c->d_export, c->export_cap, &nent))) return rc;
    std::vector<uint64_t> ent(nent * kSparseEntryWords);
    if (nent) HIPCHK(c, x_copy(c, ent.data(), c->d_export, ent.size() * 8, hipMemcpyDeviceToHost));
    size_t keep = 0;
    for (size_t i = 0; i < nent; ++i) {
      const uint64_t *w = &ent[i * kSparseEntryWords];
      const uint32_t s1 = key_s_slot1(w[0]), d1 = key_d_slot1(w[1]);
      if ((s1 < is_dead.size() && is_dead[s1]) || (d1 < is_dead.size() && is_dead[d1])) continue;
      memmove(&ent[keep * kSparseEntryWords], w, kSparseEntryWords * 8);
      ++keep;
    }
    if (keep != nent) {
      uint64_t dropped = 0;
      HIPCHK(c, x_copy(c, &dropped, c->sv.dropped, 8, hipMemcpyDeviceToHost));
      if (c->cpu) {
        cpu::sparse_init(c->sv, c->sparse_slots);
        cpu::sparse_import(c->sv, ent.data(), keep);
      } else {
        ENQ(c);
        HIPCHK(c, launch_sparse_init(c->sv, c->sparse_slots, c->stream));
        if (keep) {
          HIPCHK(c, x_copy_async(c, c->d_export, ent.data(), keep * kSparseEntryWords * 8, hipMemcpyHostToDevice,
                                   c->stream));
          ENQ(c);
          HIPCHK(c, launch_sparse_import(c->sv, c->d_export, keep, c->stream));
        }
      }
      HIPCHK(c, x_copy_async(c, c->sv.dropped, &dropped, 8, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, x_sync(c, c->stream));
    }
  }
  // the dictionary: ids become reusable
  for (uint32_t s : dead) {
    SlotAttr &a = c->slots[s];
    c->slot_ids.erase(std::make_tuple(a.ns, a.pod, a.wk_kind, a.wk_name, a.has_owner ? 1 : 0));
    a = SlotAttr();
    a.in_use = false;
    c->free_slots.push_back((int32_t)s);
  }
  ++c->slots_version;
  std::sort(c->free_slots.begin(), c->free_slots.end(), std::greater<int32_t>());  // lowest id first
  if (n_retired) *n_retired = dead.size();
  return GPUAGG_OK;
}

static std::string dns_key(uint32_t rcode, const std::string &qtypes, const std::string &query,
                           const std::string &ips, uint32_t nresp) {
  return std::to_string(rcode) + '\x1f' + qtypes + '\x1f' + query + '\x1f' + ips + '\x1f' + std::to_string(nresp);
}

// The label-canonical forms of DNS id `id` (request: qtypes, query; response: rcode name,
// qtypes, query, ips, answers): equal label tuples share one canonical id, whose label
// values are rendered once into the *_blk tables.
static void dns_canon_add(gpuagg_ctx *c, uint32_t id) {
  const DnsAttr &a = c->dns[id];
  if (c->dns_req_id.size() <= id) c->dns_req_id.resize(id + 1, 0);
  if (c->dns_resp_id.size() <= id) c->dns_resp_id.resize(id + 1, 0);
  const std::string q = a.qtypes + '\0' + a.query;
  auto i1 = c->dns_req_canon.emplace(q, (uint32_t)c->dns_req_rep.size());
  if (i1.second) {
    c->dns_req_rep.push_back(id);
    c->dns_req_blk.insert(c->dns_req_blk.end(), q.begin(), q.end());
    c->dns_req_blk.push_back('\0');
    c->dns_req_boff.push_back(c->dns_req_blk.size());
  }
  c->dns_req_id[id] = i1.first->second;
  const std::string full = std::string(a.rcode < 6 ? kRcodeNames[a.rcode] : "") + '\0' + q + '\0' + a.ips + '\0' +
                           std::to_string(a.nresp);
  auto i2 = c->dns_resp_canon.emplace(full, (uint32_t)c->dns_resp_rep.size());
  if (i2.second) {
    c->dns_resp_rep.push_back(id);
    c->dns_resp_blk.insert(c->dns_resp_blk.end(), full.begin(), full.end());
    c->dns_resp_blk.push_back('\0');
    c->dns_resp_boff.push_back(c->dns_resp_blk.size());
  }
  c->dns_resp_id[id] = i2.first->second;
}

// The canonical tables of the ids in use, from scratch (after a retire).
static void dns_canon_rebuild(gpuagg_ctx *c) {
  c->dns_req_canon.clear();
  c->dns_resp_canon.clear();
  c->dns_req_rep.clear();
  c->dns_resp_rep.clear();
  c->dns_req_blk.clear();
  c->dns_resp_blk.clear();
  c->dns_req_boff.assign(1, 0);
  c->dns_resp_boff.assign(1, 0);
  c->dns_req_rec.clear();  // the render's sort tokens: recomputed at the next snapshot
  c->dns_resp_rec.clear();
  c->dns_req_id.assign(c->dns.size(), 0);
  c->dns_resp_id.assign(c->dns.size(), 0);
  for (uint32_t id = 0; id < c->dns.size(); ++id)
    if (c->dns[id].in_use) dns_canon_add(c, id);
}

int gpuagg_dns_intern(gpuagg_ctx *c, uint32_t rcode, const char *qtypes, const char *query,
                      const char *ips, uint32_t nresp, uint32_t *id) {
  if (!c || !qtypes || !query || !ips || !id) return GPUAGG_EINVAL;
  std::string key = dns_key(rcode, qtypes, query, ips, nresp);
  auto it = c->dns_ids.find(key);
  if (it != c->dns_ids.end()) {
    c->dns[it->second].idle = false;  // handed out again: not retired at the next call
    *id = it->second;
    return GPUAGG_OK;
  }
  uint32_t nid;
  if (!c->free_dns.empty()) {  // a retired id (no group-by key references it)
    nid = c->free_dns.back();
    c->free_dns.pop_back();
    c->dns[nid] = DnsAttr{rcode, nresp, qtypes, query, ips};
  } else {
    if (c->dns.size() >= 0xFFFFFFFEull) return fail(c, GPUAGG_ECAPACITY, "DNS dictionary full");
    nid = (uint32_t)c->dns.size();
    c->dns.push_back(DnsAttr{rcode, nresp, qtypes, query, ips});
  }
  c->dns_ids.emplace(std::move(key), nid);
  dns_canon_add(c, nid);
  *id = nid;
  return GPUAGG_OK;
}

int gpuagg_dns_retire(gpuagg_ctx *const *ctxs, size_t n, uint32_t *ids, size_t cap, size_t *n_retired) {
  if (!ctxs || !n || !ctxs[0] || (cap && !ids)) return GPUAGG_EINVAL;
  gpuagg_ctx *c0 = ctxs[0];
  for (size_t i = 1; i < n; ++i) {  // one dictionary on every ctx (the producer interns alike)
    const gpuagg_ctx *ci = ctxs[i];
    if (!ci) return GPUAGG_EINVAL;
    bool same = ci->dns.size() == c0->dns.size();
    for (size_t k = 0; same && k < c0->dns.size(); ++k)
      same = ci->dns[k].in_use == c0->dns[k].in_use && ci->dns[k].rcode == c0->dns[k].rcode &&
             ci->dns[k].nresp == c0->dns[k].nresp && ci->dns[k].qtypes == c0->dns[k].qtypes &&
             ci->dns[k].query == c0->dns[k].query && ci->dns[k].ips == c0->dns[k].ips;
    if (!same) return fail(c0, GPUAGG_EINVAL, "dns_retire: ctx %zu has another DNS dictionary", i);
  }
  // ids referenced by a group-by key of a DNS family, on any ctx (after every submitted
  // batch is aggregated and every deferred list folded)
  std::vector<char> live(c0->dns.size(), 0);
  for (size_t i = 0; i < n; ++i) {
    gpuagg_ctx *c = ctxs[i];
    int rc = gpuagg_sync(c);
    if (rc) return rc;
    bool any_dns = false;
    for (const Group &g : c->groups) any_dns |= g.sparse && (g.family == FAM_DNS_REQ || g.family == FAM_DNS_RESP);
    if (!any_dns || !c->sparse_slots) continue;
    if (c->export_cap < c->sparse_slots) {
      dev_free(c, c->d_export);
      c->export_cap = 0;
      if ((rc = dev_alloc(c, &c->d_export, c->sparse_slots * kSparseEntryWords))) return rc;
      c->export_cap = c->sparse_slots;
    }
    size_t nent = 0;
    if ((rc = gpuagg_sparse_export(c, c->d_export, c->export_cap, &nent))) return rc;
    std::vector<uint64_t> ent(nent * kSparseEntryWords);
    if (nent) HIPCHK(c, x_copy(c, ent.data(), c->d_export, ent.size() * 8, hipMemcpyDeviceToHost));
    for (size_t e = 0; e < nent; ++e) {
      const uint64_t *w = &ent[e * kSparseEntryWords];
      const uint32_t grp = key_group(w[0]);
      if (grp >= c->groups.size()) continue;
      const uint8_t fam = c->groups[grp].family;
      if (fam != FAM_DNS_REQ && fam != FAM_DNS_RESP) continue;
      const uint32_t id = key_dns(w[2]);
      if (id < live.size()) live[id] = 1;
    }
  }
  // two phases: an id unreferenced now turns idle; one still unreferenced (and not handed
  // out again) at the next call is retired -- a record converted with it before this call
  // and submitted after it still finds its payload
  std::vector<uint32_t> dead, idle;
  for (uint32_t id = 0; id < c0->dns.size(); ++id) {
    if (!c0->dns[id].in_use || live[id]) continue;
    (c0->dns[id].idle ? dead : idle).push_back(id);
  }
  for (size_t i = 0; i < n; ++i) {
    gpuagg_ctx *c = ctxs[i];
    if (i && c == c0) continue;
    for (uint32_t id = 0; id < c->dns.size(); ++id) c->dns[id].idle = false;
    for (uint32_t id : idle) c->dns[id].idle = true;
    for (uint32_t id : dead) {
      DnsAttr &a = c->dns[id];
      c->dns_ids.erase(dns_key(a.rcode, a.qtypes, a.query, a.ips, a.nresp));
      a = DnsAttr{};
      a.in_use = false;
      c->free_dns.push_back(id);
    }
    std::sort(c->free_dns.begin(), c->free_dns.end(), std::greater<uint32_t>());  // lowest id first
    c->free_dns.erase(std::unique(c->free_dns.begin(), c->free_dns.end()), c->free_dns.end());
    if (!dead.empty()) dns_canon_rebuild(c);
  }
  for (size_t k = 0; k < dead.size() && k < cap; ++k) ids[k] = dead[k];
  if (n_retired) *n_retired = dead.size();
  return GPUAGG_OK;
}

int gpuagg_alloc_batch(gpuagg_ctx *c, size_t cap, gpuagg_batch **out) {
  if (!c || !out || !cap) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  auto *b = new gpuagg_batch();
  b->capacity = cap;
  for (uint32_t **p : {&b->cols.src_ip, &b->cols.dst_ip, &b->cols.bytes, &b->cols.meta,
                       &b->cols.ports, &b->cols.dns_id, &b->cols.tcp_id}) {
    if (x_host_alloc(c, (void **)p, cap * 4) != hipSuccess) {
      free_batch_cols(c, b);
      delete b;
      return fail(c, GPUAGG_ENOMEM, "hipHostMalloc(%zu)", cap * 4);
    }
    memset(*p, 0, cap * 4);
  }
  if (x_host_alloc(c, (void **)&b->cols.time_ns, cap * 8) != hipSuccess) {
    free_batch_cols(c, b);
    delete b;
    return fail(c, GPUAGG_ENOMEM, "hipHostMalloc(%zu)", cap * 8);
  }
  memset(b->cols.time_ns, 0, cap * 8);
  if (!c->cpu && (rc = ensure_staging(c, cap))) return rc;
  c->batches.push_back(b);
  *out = b;
  return GPUAGG_OK;
}

void gpuagg_free_batch(gpuagg_ctx *c, gpuagg_batch *b) {
  if (!c || !b) return;
  if (!c->cpu) {
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
  }
  free_batch_cols(c, b);
  c->batches.erase(std::remove(c->batches.begin(), c->batches.end(), b), c->batches.end());
  delete b;
}

// Enqueues the H2D copies of the columns the plan reads into the next staging buffer.
int stage_batch(gpuagg_ctx *c, const gpuagg_batch *b, size_t n, gpuagg_ctx::Staging **out, ColsView *cv) {
  int rc;
  if ((rc = ensure_staging(c, b->capacity))) return rc;
  gpuagg_ctx::Staging *s;
  if ((rc = acquire_staging(c, &s))) return rc;
  uint32_t *src[6] = {b->cols.src_ip, b->cols.dst_ip, b->cols.bytes, b->cols.meta, b->cols.ports, b->cols.dns_id};
  const bool need[6] = {true, true, (bool)c->plan.need_bytes, true, c->plan.need_ports || c->cms_len > 0,
                        (bool)c->plan.need_dns};
  for (int i = 0; i < 6; ++i)
    if (need[i] || (i == 4 && c->lat_enabled))
      HIPCHK(c, x_copy_async(c, s->cols[i], src[i], n * 4, hipMemcpyHostToDevice, c->copy_stream));
  *cv = ColsView{s->cols[0], s->cols[1], s->cols[2], s->cols[3], s->cols[4], s->cols[5]};
  if (c->lat_enabled) {
    HIPCHK(c, x_copy_async(c, s->tcp_id, b->cols.tcp_id, n * 4, hipMemcpyHostToDevice, c->copy_stream));
    HIPCHK(c, x_copy_async(c, s->time_ns, b->cols.time_ns, n * 8, hipMemcpyHostToDevice, c->copy_stream));
    cv->tcp_id = s->tcp_id;
    cv->time_ns = s->time_ns;
  }
  *out = s;
  return GPUAGG_OK;
}

int enrich_launch(gpuagg_ctx *c, const uint32_t *src, const uint32_t *dst, size_t n, int32_t *os, int32_t *od) {
  EnrichArgs a{};
  a.ip_slots = c->d_ip;
  a.ip_mask = (uint32_t)(c->ip_cap / 2 - 1);  // bucket mask
  a.ip_pre = c->radix ? c->d_rpre : nullptr;
  a.ip_blk = c->radix ? c->d_rblk : nullptr;
  a.ip_seed = c->ip_seed;
  a.src = src;
  a.dst = dst;
  a.n = n;
  a.o_src = os;
  a.o_dst = od;
  if (c->cpu) c->cpu->enrich(a);
  else {
    ENQ(c);
    HIPCHK(c, launch_enrich(a, c->n_cu, c->stream));
  }
  return GPUAGG_OK;
}

int gpuagg_submit(gpuagg_ctx *c, gpuagg_batch *b, size_t n) {
  if (!c || !b || n > b->capacity) return GPUAGG_EINVAL;
  return gpuagg::gx_submit_batch_async(c, b, n, nullptr);
}

int gpuagg_submit_enrich(gpuagg_ctx *c, gpuagg_batch *b, size_t n, int32_t *src_slot, int32_t *dst_slot) {
  if (!c || !b || n > b->capacity || !src_slot || !dst_slot) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  if (n == 0) return GPUAGG_OK;
  if (!c->ip_cap) return fail(c, GPUAGG_ESTATE, "gpuagg_set_endpoints was never called");
  if (c->cpu) {
    if ((rc = enrich_launch(c, b->cols.src_ip, b->cols.dst_ip, n, src_slot, dst_slot))) return rc;
    return launch(c, ColsView{b->cols.src_ip, b->cols.dst_ip, b->cols.bytes, b->cols.meta, b->cols.ports,
                              b->cols.dns_id, b->cols.tcp_id, b->cols.time_ns}, n);
  }
  if ((rc = ensure_buf(c, &c->d_enrich, &c->enrich_alloc, 2 * b->capacity))) return rc;
  gpuagg_ctx::Staging *s;
  ColsView cv{};
  if ((rc = stage_batch(c, b, n, &s, &cv))) return rc;
  rc = run_staged(c, *s, [&] {
    // the endpoints first, so the host copy does not wait for the aggregation
    int r = enrich_launch(c, cv.src_ip, cv.dst_ip, n, c->d_enrich, c->d_enrich + n);
    if (r) return r;
    HIPCHK(c, x_copy_async(c, src_slot, c->d_enrich, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, x_copy_async(c, dst_slot, c->d_enrich + n, n * 4, hipMemcpyDeviceToHost, c->stream));
    if ((r = launch(c, cv, n))) return r;
    // the slots are the caller's on return (the aggregation may still run)
    HIPCHK(c, hipEventRecord(c->enrich_done, c->stream));
    return GPUAGG_OK;
  });
  if (rc) return rc;
  HIPCHK(c, hipEventSynchronize(c->enrich_done));
  return GPUAGG_OK;
}

int gpuagg_submit_device(gpuagg_ctx *c, const gpuagg_columns *d, size_t n) {
  if (!c || !d) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  ColsView cv{d->src_ip, d->dst_ip, d->bytes, d->meta, d->ports, d->dns_id, d->tcp_id, d->time_ns};
  return launch(c, cv, n);
}

int gpuagg_sync(gpuagg_ctx *c) {
  if (!c) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  if ((rc = fold_pending(c))) return rc;
  // the counters come back on the stream, ahead of its one synchronisation (no blocking
  // copy per counter); the timing events are read when the stats are (gpuagg_get_stats)
  if (!c->h_sync_words) HIPCHK(c, x_host_alloc(c, (void **)&c->h_sync_words, 16));
  uint64_t *w = c->h_sync_words;
  w[0] = w[1] = 0;
  if (c->d_decode_oor) HIPCHK(c, x_copy_async(c, &w[0], c->d_decode_oor, 8, hipMemcpyDeviceToHost, c->stream));
  if (c->sparse_slots) HIPCHK(c, x_copy_async(c, &w[1], c->sv.dropped, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, x_sync(c, c->stream));
  c->stats.decode_out_of_range = w[0] + c->host_decode_oor;
  if (c->sparse_slots) c->stats.sparse_dropped = w[1];
  // an agent that keeps timing on but never reads the stats: bound the pending events
  if (c->pending_events.size() + c->pending_sketch.size() + c->pending_decode.size() + c->pending_fold.size() > 4096)
    drain_timing(c);
  return GPUAGG_OK;
}

int gpuagg_decode_device(gpuagg_ctx *c, int kind, const void *dev_raw, size_t n, const gpuagg_columns *d) {
  if (!c || !d) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  return decode(c, kind, dev_raw, n,
                OutCols{d->src_ip, d->dst_ip, d->bytes, d->meta, d->ports, d->dns_id, d->tcp_id, d->time_ns});
}

int gpuagg_submit_raw_device(gpuagg_ctx *c, int kind, const void *dev_raw, size_t n) {
  if (!c) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  if (n == 0) return GPUAGG_OK;
  if ((rc = ensure_staging(c, n))) return rc;
  gpuagg_ctx::Staging *s;
  if ((rc = acquire_staging(c, &s))) return rc;
  rc = decode_and_launch(c, *s, kind, dev_raw, n);
  if (c->cpu) return rc;
  HIPCHK(c, hipEventRecord(s->released, c->stream));
  s->in_use = true;
  return rc;
}

int gpuagg_submit_raw(gpuagg_ctx *c, int kind, const void *host_raw, size_t n) {
  if (!c || (n && !host_raw)) return GPUAGG_EINVAL;
  return gpuagg::gx_submit_raw_async(c, kind, host_raw, n, nullptr);
}

}  // extern "C"

namespace gpuagg {

int gx_submit_batch_async(gpuagg_ctx *c, gpuagg_batch *b, size_t n, hipEvent_t host_done) {
  int rc = bind(c);
  if (rc) return rc;
  if (n == 0) return GPUAGG_OK;
  if (c->cpu)  // the batch's host columns are read in place
    return launch(c, ColsView{b->cols.src_ip, b->cols.dst_ip, b->cols.bytes, b->cols.meta, b->cols.ports,
                              b->cols.dns_id, b->cols.tcp_id, b->cols.time_ns}, n);
  gpuagg_ctx::Staging *s;
  ColsView cv{};
  if ((rc = stage_batch(c, b, n, &s, &cv))) return rc;
  return run_staged(c, *s, [&] { return launch(c, cv, n); }, host_done);
}

int gx_submit_raw_async(gpuagg_ctx *c, int kind, const void *host_raw, size_t n, hipEvent_t host_done) {
  if (kind != kRawPacket && kind != kRawDrop) return fail(c, GPUAGG_EINVAL, "unknown raw record kind %d", kind);
  int rc = bind(c);
  if (rc) return rc;
  if (n == 0) return GPUAGG_OK;
  const size_t rec = kind == kRawPacket ? GPUAGG_RAW_PACKET_SIZE : GPUAGG_RAW_DROP_SIZE;
  if ((rc = ensure_staging(c, n))) return rc;
  if (c->cpu) return decode_and_launch(c, c->stg[0], kind, host_raw, n);  // decoded from the caller's memory
  gpuagg_ctx::Staging *s;
  if ((rc = acquire_staging(c, &s))) return rc;
  if (n * rec > s->raw_alloc) {  // (acquire_staging waited for the kernels reading it)
    dev_free(c, s->raw);
    s->raw_alloc = 0;
    if ((rc = dev_alloc(c, &s->raw, n * rec))) return rc;
    s->raw_alloc = n * rec;
  }
  HIPCHK(c, x_copy_async(c, s->raw, host_raw, n * rec, hipMemcpyHostToDevice, c->copy_stream));
  return run_staged(c, *s, [&] { return decode_and_launch(c, *s, kind, s->raw, n); }, host_done);
}

bool gx_is_cpu(const gpuagg_ctx *c) { return c->cpu != nullptr; }
int gx_bind(gpuagg_ctx *c) { return bind(c); }
int gx_fail(gpuagg_ctx *c, int code, const char *msg) { return fail(c, code, "%s", msg); }
int gx_host_alloc(gpuagg_ctx *c, void **p, size_t n) {
  if (int rc = bind(c)) return rc;
  if (x_host_alloc(c, p, n) != hipSuccess) return fail(c, GPUAGG_ENOMEM, "pinned host allocation (%zu bytes)", n);
  return GPUAGG_OK;
}
void gx_host_free(gpuagg_ctx *c, void *p) { x_host_free(c, p); }
int gx_prepare(gpuagg_ctx *c, size_t cap) {
  if (c->cpu) return GPUAGG_OK;
  if (int rc = bind(c)) return rc;
  return ensure_staging(c, cap);
}
uint64_t gx_time_offset(const gpuagg_ctx *c) { return (uint64_t)c->time_offset; }
void gx_count_host_decode(gpuagg_ctx *c, uint64_t n, uint64_t out_of_range) {
  c->stats.decoded += n;
  c->host_decode_oor += out_of_range;
  c->stats.decode_out_of_range += out_of_range;  // also visible before the next sync
}
void gx_feed_attach(gpuagg_ctx *c, gpuagg_raw_feed *f) { c->feeds.push_back(f); }
void gx_feed_detach(gpuagg_ctx *c, gpuagg_raw_feed *f) {
  c->feeds.erase(std::remove(c->feeds.begin(), c->feeds.end(), f), c->feeds.end());
}

}  // namespace gpuagg

extern "C" {

int gpuagg_reset(gpuagg_ctx *c) {
  if (!c) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  HIPCHK(c, x_sync(c, c->stream));
  if ((rc = lat_reset(c, false))) return rc;
  return reset_state(c);
}

namespace {
void render_latency(const gpuagg_latency_state &ls, std::map<std::string, std::string> &blocks);
}

}  // extern "C"

namespace {

// ---- snapshot rendering (the AdvancedRegistry's vectors at scrape time) ------------------
// Every counter is first reduced to a key of label-determining integer ids -- equal ids
// exactly when the rendered label strings are equal: IPs and ports are their own ids,
// pod attributes and DNS payloads are canonicalised by their strings -- so equal tuples are
// summed in hash maps on integers (partitioned over host threads) and each distinct series
// is rendered to strings once, into per-partition arenas.
void append_str(std::vector<char> &a, const char *s, size_t n) {
  const size_t o = a.size();
  a.resize(o + n + 1);
  memcpy(a.data() + o, s, n);
  a[o + n] = '\0';
}
void append_str(std::vector<char> &a, const std::string &s) { append_str(a, s.data(), s.size()); }

// Exposition sort tokens: every label value is paired with an integer whose order is its
// string's order (client_golang compares label values as strings) -- dense ranks with equal
// strings tied -- so a family's series sort on integers without touching the strings.
// run fn(t) for t < n on n threads (inline when n == 1)
template <class F>
void run_par(unsigned n, F &&fn) {
  if (n <= 1) {
    fn(0u);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < n; ++t) th.emplace_back(fn, t);
  for (auto &x : th) x.join();
}

// Sample sort on T threads: T-1 splitters from an even sample, each thread buckets its
// slice, buckets are sorted independently and land in order.
template <class E, class L>
void par_sort(std::vector<E> &v, L less, unsigned T) {
  const size_t n = v.size();
  if (T <= 1 || n < 65536) {
    std::sort(v.begin(), v.end(), less);
    return;
  }
  const size_t ov = 64;
  std::vector<E> smp;
  smp.reserve((size_t)T * ov);
  for (size_t i = 0; i < (size_t)T * ov; ++i) smp.push_back(v[i * n / ((size_t)T * ov)]);
  std::sort(smp.begin(), smp.end(), less);
  std::vector<E> sp;
  for (unsigned j = 1; j < T; ++j) sp.push_back(smp[j * ov]);
  std::vector<uint32_t> bk(n);
  std::vector<size_t> cnt((size_t)T * T, 0);  // [thread][bucket]
  run_par(T, [&](unsigned t) {
    for (size_t i = n * t / T; i < n * (t + 1) / T; ++i) {
      const uint32_t b = (uint32_t)(std::upper_bound(sp.begin(), sp.end(), v[i], less) - sp.begin());
      bk[i] = b;
      ++cnt[(size_t)t * T + b];
    }
  });
  std::vector<size_t> off((size_t)T * T), bstart(T + 1, 0);
  size_t o = 0;
  for (unsigned b = 0; b < T; ++b) {
    bstart[b] = o;
    for (unsigned t = 0; t < T; ++t) {
      off[(size_t)t * T + b] = o;
      o += cnt[(size_t)t * T + b];
    }
  }
  bstart[T] = o;
  std::vector<E> tmp(n);
  run_par(T, [&](unsigned t) {
    size_t *po = &off[(size_t)t * T];
    for (size_t i = n * t / T; i < n * (t + 1) / T; ++i) tmp[po[bk[i]]++] = v[i];
  });
  run_par(T, [&](unsigned b) { std::sort(tmp.begin() + bstart[b], tmp.begin() + bstart[b + 1], less); });
  v.swap(tmp);
}

std::vector<uint32_t> dense_ranks(const std::vector<std::string_view> &v) {
  using P = std::pair<std::string_view, uint32_t>;
  std::vector<P> ord(v.size());
  for (uint32_t i = 0; i < ord.size(); ++i) ord[i] = P{v[i], i};
  const unsigned T = (unsigned)std::min<size_t>({(size_t)16, (size_t)std::max(1u, std::thread::hardware_concurrency()),
                                                 v.size() / 16384 + 1});
  par_sort(ord, [](const P &a, const P &b) { return a.first < b.first; }, T);
  std::vector<uint32_t> rk(v.size());
  uint32_t r = 0;
  for (size_t i = 0; i < ord.size(); ++i) {
    if (i && ord[i].first != ord[i - 1].first) ++r;
    rk[ord[i].second] = r;
  }
  return rk;
}

// Fixed tables: an IPv4 label "a.b.c.d" orders as the tuple of its octets' decimal strings
// (a '.' sorts below every digit, as the string's end does), so its token is the four
// octet ranks; a port label is "unknown" (index 65536) or the port's decimal string.
struct TokTables {
  uint32_t octet[256];
  std::vector<uint32_t> port;  // 65537
  uint32_t dir_local[2], dir_remote[4], drop[16], flag[F_COUNT], rcode[7];
  TokTables() {
    std::vector<std::string> st;
    auto ranks = [&](size_t n, auto &&name) {
      st.clear();
      for (size_t i = 0; i < n; ++i) st.push_back(name(i));
      std::vector<std::string_view> sv(st.begin(), st.end());
      return dense_ranks(sv);
    };
    auto o = ranks(256, [](size_t i) { return std::to_string(i); });
    std::copy(o.begin(), o.end(), octet);
    port = ranks(65537, [](size_t i) { return i < 65536 ? std::to_string(i) : std::string("unknown"); });
    auto d = ranks(2, [](size_t i) { return std::string(i == 0 ? "ingress" : "egress"); });
    std::copy(d.begin(), d.end(), dir_local);
    d = ranks(4, [](size_t i) { return traffic_direction_name((uint32_t)i); });
    std::copy(d.begin(), d.end(), dir_remote);
    d = ranks(16, [](size_t i) { return drop_reason_name((uint32_t)i); });
    std::copy(d.begin(), d.end(), drop);
    d = ranks(F_COUNT, [](size_t i) { return std::string(kFlagNames[i]); });
    std::copy(d.begin(), d.end(), flag);
    d = ranks(7, [](size_t i) { return std::string(i < 6 ? kRcodeNames[i] : ""); });
    std::copy(d.begin(), d.end(), rcode);
  }
  uint32_t ip(uint32_t v) const {
    return octet[v & 255u] << 24 | octet[(v >> 8) & 255u] << 16 | octet[(v >> 16) & 255u] << 8 | octet[v >> 24];
  }
};
const TokTables &tok_tables() {
  static const TokTables t;
  return t;
}

// ctx_values_into's tokens, value for value
void ctx_tokens_into(const TokTables &tt, uint8_t opts, uint32_t ip, const SlotCanon &sc, uint32_t cid,
                     uint32_t port17, std::vector<uint32_t> &out) {
  if (opts & OPT_IP) out.push_back(tt.ip(ip));
  const LabelRec &lr = sc.rec[cid];
  if (opts & OPT_NS) out.push_back(lr.tok[0]);
  if (opts & OPT_POD) out.push_back(lr.tok[1]);
  if (opts & OPT_WL) {
    out.push_back(lr.tok[2]);
    out.push_back(lr.tok[3]);
  }
  if (opts & OPT_SVC) out.push_back(0u);
  if (opts & OPT_PORT) out.push_back(tt.port[(port17 & 0x10000u) ? (port17 & 0xFFFFu) : 65536u]);
}

void append_ip(std::vector<char> &out, uint32_t ip) {  // "a.b.c.d", a = the low byte
  char b[16];
  size_t n = 0;
  for (int k = 0; k < 4; ++k) {
    const uint32_t o = (ip >> (8 * k)) & 255u;
    if (k) b[n++] = '.';
    if (o >= 100) b[n++] = (char)('0' + o / 100);
    if (o >= 10) b[n++] = (char)('0' + o / 10 % 10);
    b[n++] = (char)('0' + o % 10);
  }
  append_str(out, b, n);
}
void append_port(std::vector<char> &out, uint32_t port17) {  // decimal, or "unknown"
  if (!(port17 & 0x10000u)) {
    append_str(out, "unknown", 7);
    return;
  }
  char d[8];
  int n = 0;
  uint32_t x = port17 & 0xFFFFu;
  do {
    d[7 - n++] = (char)('0' + x % 10);
    x /= 10;
  } while (x);
  append_str(out, d + 8 - n, (size_t)n);
}

// ctx_values (getByDirectionValues, types.go:418-505) into an arena.
void ctx_values_into(const gpuagg_ctx *c, uint8_t opts, uint32_t ip, uint32_t slot1, uint32_t port17,
                     std::vector<char> &out) {
  const SlotAttr *a = (slot1 && slot1 - 1 < c->slots.size()) ? &c->slots[slot1 - 1] : nullptr;
  static const std::string unk = "unknown";
  if (opts & OPT_IP) append_ip(out, ip);
  if (opts & OPT_NS) append_str(out, a ? a->ns : unk);
  if (opts & OPT_POD) append_str(out, a ? a->pod : unk);
  if (opts & OPT_WL) {
    append_str(out, a && a->has_owner ? a->wk_kind : unk);
    append_str(out, a && a->has_owner ? a->wk_name : unk);
  }
  if (opts & OPT_SVC) append_str(out, unk);
  if (opts & OPT_PORT) append_port(out, port17);
}

// ctx_values_into with the slot attributes from the canonical id's pre-rendered block
void ctx_values_fast(uint8_t opts, uint32_t ip, const SlotCanon &sc, uint32_t cid, uint32_t port17,
                     std::vector<char> &out) {
  if (opts & OPT_IP) append_ip(out, ip);
  if (opts & (OPT_NS | OPT_POD | OPT_WL)) {
    const LabelRec &lr = sc.rec[cid];
    out.insert(out.end(), sc.blk.data() + lr.off, sc.blk.data() + lr.off + lr.len);
  }
  if (opts & OPT_SVC) append_str(out, "unknown", 7);
  if (opts & OPT_PORT) append_port(out, port17);
}

int render_series(gpuagg_ctx *c, const std::vector<uint64_t> &dc, const std::vector<uint64_t> &db,
                  const std::vector<uint64_t> &ent, size_t nent, gpuagg_result *r) {
  const bool local = !c->remote;
  const size_t ns_len = strlen("networkobservability_");
  r->fam.resize(c->inst.size());
  for (size_t ii = 0; ii < c->inst.size(); ++ii) {
    ResultFamily &f = r->fam[ii];
    const Instance &in = c->inst[ii];
    const FamilyInfo fi = family_info(in.vec_name.substr(ns_len));
    f.metric = in.vec_name;
    f.names = in.label_names;
    f.type = fi.type;
    f.help = fi.help;
  }
  for (auto &f : r->fam) {  // (pointers taken once the vector is final)
    for (auto &n : f.names) f.name_ptrs.push_back(n.c_str());
    f.by_name.resize(f.names.size());
    for (uint32_t k = 0; k < f.by_name.size(); ++k) f.by_name[k] = k;
    std::stable_sort(f.by_name.begin(), f.by_name.end(),
                     [&](uint32_t a, uint32_t b) { return f.names[a] < f.names[b]; });
  }
  // views: (group, src labels, dst labels) of the active instances
  struct View {
    int group;
    bool src, dst;
    std::vector<uint32_t> insts;
  };
  std::vector<View> views;
  std::vector<std::vector<uint32_t>> group_views(c->groups.size());
  for (size_t ii = 0; ii < c->inst.size(); ++ii) {
    const Instance &in = c->inst[ii];
    if (!in.active || in.group < 0) continue;
    const bool s = local || in.has_src, d = !local && in.has_dst;
    uint32_t v = 0;
    while (v < views.size() && !(views[v].group == in.group && views[v].src == s && views[v].dst == d)) ++v;
    if (v == views.size()) {
      views.push_back(View{in.group, s, d, {}});
      group_views[in.group].push_back(v);
    }
    views[v].insts.push_back((uint32_t)ii);
  }
  if (views.empty()) return GPUAGG_OK;
  // canonical slot attributes per option mask (cached until the slots change)
  std::map<uint8_t, SlotCanon> &canon = c->slot_canon;
  auto slot_canon = [&](uint8_t opts) -> const SlotCanon & {
    const uint8_t m = opts & (OPT_NS | OPT_POD | OPT_WL);
    SlotCanon &sc = canon[m];
    if (sc.version == c->slots_version) return sc;
    sc.id.assign(c->slots.size() + 1, 0u);
    sc.rep.clear();
    if (!(m & (OPT_NS | OPT_POD | OPT_WL))) {  // nothing slot-derived: one id
      sc.rep.push_back(0u);
    } else {
      std::unordered_map<std::string, uint32_t> ids;
      ids.reserve(c->slots.size() + 1);
      std::vector<char> buf;
      for (uint32_t s1 = 0; s1 <= c->slots.size(); ++s1) {
        buf.clear();
        ctx_values_into(c, m, 0, s1, 0, buf);
        auto ins = ids.emplace(std::string(buf.begin(), buf.end()), (uint32_t)sc.rep.size());
        if (ins.second) sc.rep.push_back(s1);
        sc.id[s1] = ins.first->second;
      }
    }
    sc.blk.clear();
    sc.rec.assign(sc.rep.size(), LabelRec{});
    for (size_t i = 0; i < sc.rep.size(); ++i) {
      sc.rec[i].off = sc.blk.size();
      ctx_values_into(c, m, 0, sc.rep[i], 0, sc.blk);
      sc.rec[i].len = (uint32_t)(sc.blk.size() - sc.rec[i].off);
    }
    static const std::string unk = "unknown";
    for (int f = 0; f < 4; ++f) {
      std::vector<std::string_view> sv(sc.rep.size());
      for (size_t i = 0; i < sc.rep.size(); ++i) {
        const uint32_t s1 = sc.rep[i];
        const SlotAttr *a = (s1 && s1 - 1 < c->slots.size()) ? &c->slots[s1 - 1] : nullptr;
        const std::string *x = &unk;
        if (a && f == 0) x = &a->ns;
        if (a && f == 1) x = &a->pod;
        if (a && a->has_owner && f == 2) x = &a->wk_kind;
        if (a && a->has_owner && f == 3) x = &a->wk_name;
        sv[i] = *x;
      }
      const std::vector<uint32_t> rk = dense_ranks(sv);
      for (size_t i = 0; i < sc.rep.size(); ++i) sc.rec[i].tok[f] = rk[i];
    }
    sc.version = c->slots_version;
    return sc;
  };
  for (const View &v : views) {
    slot_canon(c->groups[v.group].src_opts);
    slot_canon(c->groups[v.group].dst_opts);
  }
  auto cid = [&](const SlotCanon &sc, uint32_t slot1) { return sc.id[slot1 < sc.id.size() ? slot1 : 0]; };
  // each viewed group's canonical tables, looked up once
  std::vector<const SlotCanon *> src_canon(c->groups.size(), nullptr), dst_canon(c->groups.size(), nullptr);
  for (const View &v : views) {
    const Group &g = c->groups[v.group];
    src_canon[v.group] = &canon.at(g.src_opts & (OPT_NS | OPT_POD | OPT_WL));
    dst_canon[v.group] = &canon.at(g.dst_opts & (OPT_NS | OPT_POD | OPT_WL));
  }
  // canonical DNS payloads (kept by gpuagg_dns_intern)
  const std::vector<uint32_t> &dns_req = c->dns_req_id, &dns_resp = c->dns_resp_id;
  const std::vector<uint32_t> &dns_req_rep = c->dns_req_rep, &dns_resp_rep = c->dns_resp_rep;
  const TokTables &tt = tok_tables();
  bool any_dns = false;
  for (const View &v : views)
    any_dns |= c->groups[v.group].family == FAM_DNS_REQ || c->groups[v.group].family == FAM_DNS_RESP;
  auto dns_recs = [&](std::vector<LabelRec> &rec, const std::vector<uint32_t> &reps,
                      const std::vector<uint64_t> &boff, bool resp) {
    if (rec.size() == reps.size()) return;  // (tokens are recomputed as the table grows)
    const size_t n = reps.size();
    rec.assign(n, LabelRec{});
    for (size_t i = 0; i < n; ++i) {
      rec[i].off = boff[i];
      rec[i].len = (uint32_t)(boff[i + 1] - boff[i]);
    }
    std::vector<std::string_view> sv(n);
    std::vector<std::string> nr;
    auto field = [&](int f, auto &&get) {
      for (size_t i = 0; i < n; ++i) sv[i] = get(c->dns[reps[i]], i);
      const std::vector<uint32_t> rk = dense_ranks(sv);
      for (size_t i = 0; i < n; ++i) rec[i].tok[f] = rk[i];
    };
    int f = 0;
    if (resp)
      for (size_t i = 0; i < n; ++i) rec[i].tok[f] = tt.rcode[std::min<uint32_t>(c->dns[reps[i]].rcode, 6u)];
    f += resp;
    field(f++, [](const DnsAttr &a, size_t) -> std::string_view { return a.qtypes; });
    field(f++, [](const DnsAttr &a, size_t) -> std::string_view { return a.query; });
    if (resp) {
      field(f++, [](const DnsAttr &a, size_t) -> std::string_view { return a.ips; });
      nr.resize(n);
      for (size_t i = 0; i < n; ++i) nr[i] = std::to_string(c->dns[reps[i]].nresp);
      field(f++, [&](const DnsAttr &, size_t i) -> std::string_view { return nr[i]; });
    }
  };
  if (any_dns) {
    dns_recs(c->dns_req_rec, dns_req_rep, c->dns_req_boff, false);
    dns_recs(c->dns_resp_rec, dns_resp_rep, c->dns_resp_boff, true);
  }
  // items: one per (counter, view), partitioned by key hash
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t work = nent + (size_t)c->dense_len;
  const unsigned T = (unsigned)std::max<size_t>(1, std::min<size_t>({(size_t)16, (size_t)hw, work / 65536 + 1}));
  // (the ctx's scratch: kept between snapshots, so its pages stay faulted in)
  auto &parts = c->agg_scratch.parts;
  if (parts.size() < T) parts.resize(T);
  for (unsigned t = 0; t < T; ++t) {
    if (parts[t].size() < T) parts[t].resize(T);
    for (unsigned q = 0; q < T; ++q) parts[t][q].clear();
  }
  std::vector<int> err(T, GPUAGG_OK);
  std::vector<uint64_t> dead_dns(T, 0);  // entries of retired DNS ids: not rendered, counted as lost
  auto run = [&](auto &&fn) {  // fn(t) on T threads
    if (T == 1) {
      fn(0u);
      return;
    }
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; ++t) th.emplace_back(fn, t);
    for (auto &x : th) x.join();
  };
  auto put = [&](unsigned t, const LKey &k, uint64_t cn, uint64_t by) {
    parts[t][LKeyHash()(k) % T].push_back(LItem{k, cn, by});
  };
  run([&](unsigned t) {
    // sparse entries [t * nent / T, (t + 1) * nent / T)
    const size_t e0 = nent * t / T, e1 = nent * (t + 1) / T;
    for (size_t e = e0; e < e1; ++e) {
      const uint64_t *w = &ent[e * kSparseEntryWords];
      const uint32_t grp = key_group(w[0]);
      if (grp >= group_views.size()) continue;
      const Group &g = c->groups[grp];
      const uint32_t sub = key_sub(w[0]);
      const uint32_t hi = sub >> 3, tdir = (sub >> 1) & 3, side = sub & 1;
      const uint32_t dirv = local ? side : tdir;
      uint32_t pre = 0;
      switch (g.family) {
        case FAM_FWD:
        case FAM_RETRANS: pre = dirv; break;
        case FAM_DROP: pre = (hi << 4) | dirv; break;
        case FAM_TCPFLAGS: pre = hi; break;
        case FAM_DNS_REQ:
        case FAM_DNS_RESP: {
          const uint32_t id = key_dns(w[2]);
          if (id < c->dns.size() && !c->dns[id].in_use) {  // a retired id in a late record
            ++dead_dns[t];
            continue;
          }
          if (id >= c->dns.size()) {
            err[t] = GPUAGG_EINVAL;
            return;
          }
          pre = g.family == FAM_DNS_REQ ? dns_req[id] : dns_resp[id];
          break;
        }
      }
      for (uint32_t vi : group_views[grp]) {
        const View &v = views[vi];
        LKey k{};
        k.w[0] = vi;
        k.w[1] = pre;
        if (v.src) {
          k.w[2] = (g.src_opts & OPT_IP) ? key_s_ip(w[0]) : 0u;
          k.w[3] = cid(*src_canon[grp], key_s_slot1(w[0]));
          k.w[4] = (g.src_opts & OPT_PORT) ? key_s_port17(w[1]) : 0u;
        }
        if (v.dst) {
          k.w[5] = (g.dst_opts & OPT_IP) ? key_d_ip(w[2]) : 0u;
          k.w[6] = cid(*dst_canon[grp], key_d_slot1(w[1]));
          k.w[7] = (g.dst_opts & OPT_PORT) ? key_d_port17(w[1]) : 0u;
        }
        put(t, k, w[3], w[4]);
      }
    }
    // dense bins: group by group, keys split over the threads
    for (size_t gi = 0; gi < c->groups.size(); ++gi) {
      const Group &g = c->groups[gi];
      if (g.sparse || group_views[gi].empty()) continue;
      const SlotCanon &sc = *src_canon[gi];
      const uint64_t k0 = g.nkeys * t / T, k1 = g.nkeys * (t + 1) / T;
      for (uint64_t key = k0; key < k1; ++key)
        for (uint32_t side = 0; side < 2; ++side)
          for (uint32_t sub = 0; sub < g.nsub; ++sub) {
            const uint64_t idx = g.dense_base + (key * 2 + side) * g.nsub + sub;
            if (!dc[idx]) continue;  // (a bytes series exists whenever its count does)
            const uint32_t pre = g.family == FAM_DROP ? (sub << 4) | side : g.family == FAM_TCPFLAGS ? sub : side;
            for (uint32_t vi : group_views[gi]) {
              LKey k{};
              k.w[0] = vi;
              k.w[1] = pre;
              k.w[3] = cid(sc, g.key_mode ? (uint32_t)key + 1 : 0u);
              put(t, k, dc[idx], db[idx]);
            }
          }
    }
  });
  for (int e : err)
    if (e) return fail(c, e, "snapshot: a group-by key names a dns_id that was not interned");
  for (uint64_t d : dead_dns) r->dropped += d;
  // per partition: sum equal keys, then render each distinct key's series into the
  // partition's arena
  auto &out = c->agg_scratch.out;
  auto &tabs = c->agg_scratch.tab;
  if (out.size() < T) out.resize(T);
  if (tabs.size() < T) tabs.resize(T);
  for (unsigned p = 0; p < T; ++p) out[p].clear();
  r->pool = c->scrape_pool;
  {  // the pool's arenas / token lists (capacity kept), fresh ones past them
    std::lock_guard<std::mutex> lk(r->pool->mu);
    r->arenas.resize(T);
    r->toks.resize(T);
    for (unsigned p = 0; p < T; ++p) {
      if (!r->pool->arenas.empty()) {
        r->arenas[p].swap(r->pool->arenas.back());
        r->pool->arenas.pop_back();
      }
      if (!r->pool->toks.empty()) {
        r->toks[p].swap(r->pool->toks.back());
        r->pool->toks.pop_back();
      }
      r->arenas[p].clear();
      r->toks[p].clear();
    }
    r->series.swap(r->pool->series);
    r->series.clear();
  }
  run([&](unsigned p) {
    size_t total = 0;
    for (unsigned t = 0; t < T; ++t) total += parts[t][p].size();
    // open addressing (linear probing, at most half full); w[0] (the view) is never ~0
    size_t cap = 16;
    while (cap < 2 * total) cap <<= 1;
    std::vector<LItem> &tab = tabs[p];
    if (tab.size() < cap) tab.resize(cap);
    for (size_t i = 0; i < cap; ++i) tab[i].k.w[0] = ~0u;
    size_t NM = 0;
    for (unsigned t = 0; t < T; ++t) {
      for (const LItem &it : parts[t][p]) {
        size_t h = fmix64(LKeyHash()(it.k)) & (cap - 1);
        while (tab[h].k.w[0] != ~0u && !(tab[h].k == it.k)) h = (h + 1) & (cap - 1);
        LItem &e = tab[h];
        if (e.k.w[0] == ~0u) {
          e = it;
          ++NM;
        } else {
          e.cnt += it.cnt;
          e.byt += it.byt;
        }
      }
      parts[t][p].clear();
    }
    std::vector<char> &ar = r->arenas[p];
    std::vector<uint32_t> &tk = r->toks[p];
    // (reserved generously: pages never written are never faulted in)
    ar.reserve(NM * 320);
    tk.reserve(NM * 16);
    out[p].reserve(NM * 2);
    for (size_t ti = 0; ti < cap; ++ti) {  // (the reused table may be longer than cap)
      const LItem &kv = tab[ti];
      if (kv.k.w[0] == ~0u) continue;
      const LKey &k = kv.k;
      const View &v = views[k.w[0]];
      const Group &g = c->groups[v.group];
      // the view's instances (count / bytes objects) share the labels: rendered once
      const uint64_t off = ar.size(), tok = tk.size();
      const uint32_t pre = k.w[1];
      auto dir = [&](uint32_t d) {
        if (local) {
          append_str(ar, d == 0 ? "ingress" : "egress", d == 0 ? 7 : 6);
          tk.push_back(tt.dir_local[d & 1u]);
        } else {
          append_str(ar, traffic_direction_name(d));
          tk.push_back(tt.dir_remote[d & 3u]);
        }
      };
      switch (g.family) {
        case FAM_FWD:
        case FAM_RETRANS: dir(pre); break;
        case FAM_DROP:
          append_str(ar, drop_reason_name(pre >> 4));
          tk.push_back(tt.drop[(pre >> 4) & 15u]);
          dir(pre & 15u);
          break;
        case FAM_TCPFLAGS:
          append_str(ar, kFlagNames[pre]);
          tk.push_back(tt.flag[pre]);
          break;
        case FAM_DNS_REQ:
        case FAM_DNS_RESP: {
          if (g.family == FAM_DNS_REQ) {  // qtypes, query
            const LabelRec &lr = c->dns_req_rec[pre];
            ar.insert(ar.end(), c->dns_req_blk.data() + lr.off, c->dns_req_blk.data() + lr.off + lr.len);
            tk.insert(tk.end(), lr.tok, lr.tok + 2);
          } else {  // rcode, qtypes, query, ips, answers
            const LabelRec &lr = c->dns_resp_rec[pre];
            ar.insert(ar.end(), c->dns_resp_blk.data() + lr.off, c->dns_resp_blk.data() + lr.off + lr.len);
            tk.insert(tk.end(), lr.tok, lr.tok + 5);
          }
          break;
        }
      }
      if (v.src) {
        ctx_values_fast(g.src_opts, k.w[2], *src_canon[v.group], k.w[3], k.w[4], ar);
        ctx_tokens_into(tt, g.src_opts, k.w[2], *src_canon[v.group], k.w[3], k.w[4], tk);
      }
      if (v.dst) {
        ctx_values_fast(g.dst_opts, k.w[5], *dst_canon[v.group], k.w[6], k.w[7], ar);
        ctx_tokens_into(tt, g.dst_opts, k.w[5], *dst_canon[v.group], k.w[6], k.w[7], tk);
      }
      const uint32_t len = (uint32_t)(ar.size() - off);
      const char *b = ar.data() + off;
      const uint32_t esc = memchr(b, '\\', len) || memchr(b, '"', len) || memchr(b, '\n', len);
      for (uint32_t ii : v.insts)
        out[p].push_back(SeriesRec{ii, p, off, c->inst[ii].vk == VK_BYTES ? kv.byt : kv.cnt, tok,
                                   len, esc});
    }
  });
  // concatenate the partitions
  std::vector<size_t> sbase(T + 1, 0);
  for (unsigned p = 0; p < T; ++p) sbase[p + 1] = sbase[p] + out[p].size();
  r->series.resize(sbase[T]);
  run([&](unsigned p) {
    std::copy(out[p].begin(), out[p].end(), r->series.begin() + sbase[p]);
    out[p].clear();
  });
  return GPUAGG_OK;
}

}  // namespace

extern "C" {

int gpuagg_snapshot(gpuagg_ctx *c, gpuagg_result **out) {
  if (!c || !out) return GPUAGG_EINVAL;
  *out = nullptr;
  int rc = gpuagg_sync(c);
  if (rc) return rc;

  // dense counters
  std::vector<uint64_t> dc(c->dense_len), db(c->dense_len);
  if (c->dense_len) {
    HIPCHK(c, x_copy(c, dc.data(), c->d_dense_cnt, c->dense_len * 8, hipMemcpyDeviceToHost));
    HIPCHK(c, x_copy(c, db.data(), c->d_dense_byt, c->dense_len * 8, hipMemcpyDeviceToHost));
  }
  // sparse entries
  std::vector<uint64_t> ent;
  size_t nent = 0;
  if (c->sparse_slots) {
    uint64_t dropped = 0;
    HIPCHK(c, x_copy(c, &dropped, c->sv.dropped, 8, hipMemcpyDeviceToHost));
    c->stats.sparse_dropped = dropped;  // reported with the result (gpuagg_result_dropped)
    if (c->export_cap < c->sparse_slots) {
      dev_free(c, c->d_export);
      if ((rc = dev_alloc(c, &c->d_export, c->sparse_slots * kSparseEntryWords))) return rc;
      c->export_cap = c->sparse_slots;
    }
    rc = gpuagg_sparse_export(c, c->d_export, c->export_cap, &nent);
    if (rc) return rc;
    ent.resize(nent * kSparseEntryWords);
    if (nent) HIPCHK(c, x_copy(c, ent.data(), c->d_export, ent.size() * 8, hipMemcpyDeviceToHost));
    c->stats.sparse_entries = nent;
  }

  auto *r = new gpuagg_result();
  r->dropped = c->stats.sparse_dropped;
  if ((rc = render_series(c, dc, db, ent, nent, r))) {
    gpuagg_result_free(r);
    return rc;
  }
  if (c->cms_len || c->hll_len) {
    if ((rc = gpuagg_sketch_refresh(c))) {
      gpuagg_result_free(r);
      return rc;
    }
  }
  if (c->lat_enabled) {
    gpuagg_latency_state ls{};
    if ((rc = gpuagg_latency_read(c, &ls))) {
      gpuagg_result_free(r);
      return rc;
    }
    render_latency(ls, r->extra_text);
  }
  *out = r;
  return GPUAGG_OK;
}

size_t gpuagg_result_count(const gpuagg_result *r) { return r ? r->series.size() : 0; }

int gpuagg_result_family(const gpuagg_result *r, size_t i, const char **type, const char **help) {
  if (!r || i >= r->series.size()) return GPUAGG_EINVAL;
  if (type) *type = r->fam[r->series[i].fam].type;
  if (help) *help = r->fam[r->series[i].fam].help;
  return GPUAGG_OK;
}

uint64_t gpuagg_result_dropped(const gpuagg_result *r) { return r ? r->dropped : 0; }

namespace {
// Go strconv.FormatFloat(v, 'g', -1, 64), as expfmt writes a sample value: the shortest
// decimal digits d1.d2..dn x 10^x that round-trip, in %e form (exponent of at least two
// digits) when x < -4 or x >= 6 -- Go's fmtG uses precision 6 for that choice when the
// digits are the shortest (strconv/ftoa.go) -- else in %f form.
std::string go_float_g(double v);

// go_float_g of an exact integer count: below 2^53 every integer is a double of its own
// and a decimal with fewer significant digits is another integer, so the shortest
// round-trip digits are the integer's, trailing zeros dropped (no probing).
void go_float_u64_into(std::string &out, uint64_t v) {
  if (v > (1ULL << 53)) {
    out += go_float_g((double)v);
    return;
  }
  char d[24];
  int n = 0;
  do {
    d[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  const int x = n - 1;  // decimal exponent; digits most significant first: d[n-1] .. d[0]
  if (x < 6) {          // Go 'g', shortest: %e only from exponent 6 (ftoa.go eprec = 6)
    for (int k = n - 1; k >= 0; --k) out += d[k];
    return;
  }
  int lo = 0;
  while (lo < n - 1 && d[lo] == '0') ++lo;  // trailing zeros
  out += d[n - 1];
  if (n - 1 > lo) {
    out += '.';
    for (int k = n - 2; k >= lo; --k) out += d[k];
  }
  char e[8];
  snprintf(e, sizeof e, "e+%02d", x);
  out += e;
}

std::string go_float_g(double v) {
  if (v == 0) return "0";
  char buf[64];
  // shortest round-trip digits via %.17g probing
  int prec = 1;
  for (; prec <= 17; ++prec) {
    snprintf(buf, sizeof buf, "%.*e", prec - 1, v);
    if (strtod(buf, nullptr) == v) break;
  }
  // buf = d.ddde[+-]XX
  std::string m(buf);
  const size_t epos = m.find('e');
  const int x = atoi(m.c_str() + epos + 1);
  std::string digits;
  for (size_t k = 0; k < epos; ++k)
    if (isdigit((unsigned char)m[k])) digits += m[k];
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  const bool neg = v < 0;
  // Go: shortest => eprec = 6; "%e is used if the exponent from the conversion is less
  // than -4 or greater than or equal to the precision"; if eprec > digits and digits >=
  // decimal point position, eprec = digits ... with shortest it is 6 (ftoa.go)
  int eprec = 6;
  std::string out = neg ? "-" : "";
  if (x < -4 || x >= eprec) {
    out += digits[0];
    if (digits.size() > 1) {
      out += '.';
      out += digits.substr(1);
    }
    char e[16];
    snprintf(e, sizeof e, "e%c%02d", x < 0 ? '-' : '+', x < 0 ? -x : x);
    out += e;
    return out;
  }
  if (x >= 0) {  // integer part digits[0..x], fraction the rest
    std::string ip = digits.substr(0, std::min<size_t>(digits.size(), (size_t)x + 1));
    while ((int)ip.size() < x + 1) ip += '0';
    out += ip;
    if (digits.size() > (size_t)x + 1) out += "." + digits.substr(x + 1);
  } else {
    out += "0." + std::string((size_t)(-x - 1), '0') + digits;
  }
  return out;
}

// Latency families (latency.go:28-33, LinearBuckets(0, 0.5, 10)): histograms as
// cumulative le buckets + _sum + _count, no_response once its vec child exists.
void render_latency(const gpuagg_latency_state &ls, std::map<std::string, std::string> &blocks) {
  auto hist = [&](const char *name, const char *help, const uint64_t *bk, uint64_t cnt, int64_t sum) {
    std::string &o = blocks[name];
    o += std::string("# HELP ") + name + " " + help + "\n# TYPE " + name + " histogram\n";
    uint64_t acc = 0;
    for (int i = 0; i < 11; ++i) {
      acc += bk[i];
      o += std::string(name) + "_bucket{le=\"" + (i == 10 ? std::string("+Inf") : go_float_g(0.5 * i)) + "\"} " +
           std::to_string(acc) + "\n";
    }
    o += std::string(name) + "_sum " + go_float_g((double)sum) + "\n";
    o += std::string(name) + "_count " + std::to_string(cnt) + "\n";
  };
  if (ls.enabled & 1u)
    hist("networkobservability_adv_node_apiserver_latency", "Latency of node apiserver in ms",
         ls.latency_buckets, ls.latency_count, ls.latency_sum);
  if (ls.enabled & 2u)
    hist("networkobservability_adv_node_apiserver_tcp_handshake_latency",
         "Latency of node apiserver tcp handshake in ms", ls.handshake_buckets, ls.handshake_count,
         ls.handshake_sum);
  if ((ls.enabled & 4u) && ls.no_response) {
    const char *name = "networkobservability_adv_node_apiserver_no_response";
    blocks[name] = std::string("# HELP ") + name +
                   " Number of packets that did not get a response from node apiserver\n# TYPE " + name +
                   " counter\n" + name + "{no_response=\"no_response\"} " + go_float_g((double)ls.no_response) + "\n";
  }
}

void escape_cstr(std::string &out, const char *s, bool quote) {  // expfmt escaping
  const size_t n = strlen(s);
  if (!memchr(s, '\\', n) && !memchr(s, '\n', n) && !(quote && memchr(s, '"', n))) {
    out.append(s, n);  // nothing to escape (the usual case)
    return;
  }
  for (; *s; ++s) {
    const char ch = *s;
    if (ch == '\\') out += "\\\\";
    else if (ch == '\n') out += "\\n";
    else if (quote && ch == '"') out += "\\\"";
    else out += ch;
  }
}
void escape_into(std::string &out, const std::string &s, bool quote) { escape_cstr(out, s.c_str(), quote); }


// Series of one family in exposition order (client_golang sorts a family's metrics by
// their label values taken in label-name order; MetricSorter), on the values' sort tokens
// (render_series): packed into one 128-bit key when their widths fit, else as rows.
void sort_family(const gpuagg_result *r, const ResultFamily &F, std::vector<size_t> &idx, unsigned T,
                 std::vector<uint32_t> &perm) {
  const size_t n = idx.size(), nl = F.names.size();
  perm.resize(n);
  for (size_t q = 0; q < n; ++q) perm[q] = (uint32_t)q;
  if (n < 2 || nl == 0) return;
  std::vector<uint32_t> rk(n * nl);  // tokens in name order
  std::vector<std::vector<uint32_t>> mx(T, std::vector<uint32_t>(nl, 0));
  run_par(T, [&](unsigned t) {
    for (size_t q = n * t / T; q < n * (t + 1) / T; ++q) {
      const SeriesRec &sr = r->series[idx[q]];
      const uint32_t *tok = r->toks[sr.arena].data() + sr.tok;
      for (size_t k = 0; k < nl; ++k) {
        const uint32_t x = tok[F.by_name[k]];
        rk[q * nl + k] = x;
        mx[t][k] = std::max(mx[t][k], x);
      }
    }
  });
  std::vector<unsigned> bits(nl, 0);
  unsigned tbits = 0;
  for (size_t k = 0; k < nl; ++k) {
    uint32_t m = 0;
    for (unsigned t = 0; t < T; ++t) m = std::max(m, mx[t][k]);
    while (bits[k] < 32 && (m >> bits[k])) ++bits[k];
    tbits += bits[k];
  }
  if (tbits <= 128) {
    using K = std::pair<unsigned __int128, uint32_t>;
    std::vector<K> keys(n);
    run_par(T, [&](unsigned t) {
      for (size_t q = n * t / T; q < n * (t + 1) / T; ++q) {
        unsigned __int128 x = 0;
        for (size_t k = 0; k < nl; ++k) x = (x << bits[k]) | rk[q * nl + k];
        keys[q] = K{x, (uint32_t)q};
      }
    });
    par_sort(keys, [](const K &a, const K &b) { return a.first < b.first; }, T);
    for (size_t q = 0; q < n; ++q) perm[q] = keys[q].second;
  } else {
    std::vector<uint32_t> ord(n);
    for (size_t q = 0; q < n; ++q) ord[q] = (uint32_t)q;
    par_sort(ord, [&](uint32_t a, uint32_t b) {
      const uint32_t *x = &rk[(size_t)a * nl], *y = &rk[(size_t)b * nl];
      for (size_t k = 0; k < nl; ++k)
        if (x[k] != y[k]) return x[k] < y[k];
      return false;
    }, T);
    perm = std::move(ord);
  }
  const std::vector<size_t> old = idx;
  for (size_t q = 0; q < n; ++q) idx[q] = old[perm[q]];
}

// expfmt escaping of a label value into a raw buffer sized for the worst case (2x)
inline char *escape_raw(char *o, const char *s) {
  for (; *s; ++s) {
    const char ch = *s;
    if (ch == '\\' || ch == '"') {
      *o++ = '\\';
      *o++ = ch;
    } else if (ch == '\n') {
      *o++ = '\\';
      *o++ = 'n';
    } else {
      *o++ = ch;
    }
  }
  return o;
}

// Label values of a series, in label order, from its arena block (NUL-separated).
inline void series_values(const gpuagg_result *r, const SeriesRec &sr, size_t nl, const char **v) {
  const char *q = r->arenas[sr.arena].data() + sr.off;
  for (size_t j = 0; j < nl; ++j) {
    v[j] = q;
    q += strlen(q) + 1;
  }
}

void build_value_ptrs(const gpuagg_result *r) {
  const size_t ns = r->series.size();
  r->voff.resize(ns + 1);
  uint64_t nv = 0;
  for (size_t i = 0; i < ns; ++i) {
    r->voff[i] = nv;
    nv += r->fam[r->series[i].fam].names.size();
  }
  r->voff[ns] = nv;
  r->value_ptrs.resize(nv);
  const unsigned T = (unsigned)std::max<size_t>(1, std::min<size_t>({(size_t)16, (size_t)std::max(1u, std::thread::hardware_concurrency()),
                                                                    ns / 65536 + 1}));
  run_par(T, [&](unsigned t) {
    for (size_t i = ns * t / T; i < ns * (t + 1) / T; ++i)
      series_values(r, r->series[i], r->voff[i + 1] - r->voff[i], r->value_ptrs.data() + r->voff[i]);
  });
}

// A sample value as expfmt writes it (go_float_u64_into) at w; returns its length.
inline size_t put_value(char *w, uint64_t x) {
  if (x < 1000000) {  // plain integer digits (go_float_u64_into's short case)
    char d[8];
    size_t m = 0;
    do {
      d[m++] = (char)('0' + x % 10);
      x /= 10;
    } while (x);
    for (size_t k = 0; k < m; ++k) w[k] = d[m - 1 - k];
    return m;
  }
  std::string f;
  go_float_u64_into(f, x);
  memcpy(w, f.data(), f.size());
  return f.size();
}

inline size_t escaped_len(const char *s) {
  size_t e = 0;
  for (; *s; ++s) e += 1 + (*s == '\\' || *s == '"' || *s == '\n');
  return e;
}

// gpuagg_result_render_text's text, built once per result: families sorted by name
// (expfmt), each family's series in client_golang's order.  Every series' exact length is
// known first (its label bytes from render_series), so the threads write straight into
// the final buffer at their offsets.
void render_text(const gpuagg_result *r) {
  std::vector<std::vector<size_t>> by_fam(r->fam.size());
  for (size_t i = 0; i < r->series.size(); ++i) by_fam[r->series[i].fam].push_back(i);
  std::map<std::string, size_t> fam;  // metric name -> family
  for (size_t f = 0; f < by_fam.size(); ++f)
    if (!by_fam[f].empty()) fam[r->fam[f].metric] = f;
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  // families whose series share their labels series for series (the count and bytes
  // objects of one view): sorted once, the partner takes the same permutation
  std::vector<int> partner(r->fam.size(), -1);
  for (size_t f = 0; f < by_fam.size(); ++f)
    for (size_t g = 0; g < f && partner[f] < 0; ++g) {
      if (by_fam[g].size() != by_fam[f].size() || by_fam[f].empty() || r->fam[g].names != r->fam[f].names) continue;
      bool same = true;
      for (size_t q = 0; same && q < by_fam[f].size(); ++q) {
        const SeriesRec &a = r->series[by_fam[f][q]], &b = r->series[by_fam[g][q]];
        same = a.arena == b.arena && a.off == b.off;
      }
      if (same) partner[f] = (int)g;
    }
  std::vector<std::vector<uint32_t>> perms(r->fam.size());
  struct Job {
    const std::string *text = nullptr;  // a fixed block (extra family, header) ...
    std::string own;
    size_t f = 0;  // ... or family f's series
    unsigned T = 1;
    std::vector<std::string> lab;
    std::vector<uint64_t> at;  // series q's offset within the job (n + 1)
    uint64_t base = 0, size = 0;
  };
  std::vector<Job> jobs;
  std::map<std::string, int> names;  // every family name, extra blocks included
  for (auto &kv : r->extra_text) names[kv.first] = 0;
  for (auto &kv : fam) names[kv.first] = 0;
  for (auto &nk : names) {
    auto ex = r->extra_text.find(nk.first);
    if (ex != r->extra_text.end()) {
      jobs.emplace_back();
      jobs.back().text = &ex->second;
      jobs.back().size = ex->second.size();
    }
    auto fi = fam.find(nk.first);
    if (fi == fam.end()) continue;
    const size_t f = fi->second;
    std::vector<size_t> &idx = by_fam[f];
    const ResultFamily &F = r->fam[f];
    const size_t nl = F.names.size(), n = idx.size();
    jobs.emplace_back();
    Job &h = jobs.back();
    h.own = "# HELP " + nk.first + " ";
    escape_cstr(h.own, F.help, false);
    h.own += "\n# TYPE " + nk.first + " " + F.type + "\n";
    h.size = h.own.size();
    jobs.emplace_back();
    Job &j = jobs.back();
    j.f = f;
    j.T = (unsigned)std::max<size_t>(1, std::min<size_t>({(size_t)16, (size_t)hw, n / 8192 + 1}));
    const int pg = partner[f] >= 0 ? partner[f] : -1;
    int done = -1;  // a sorted family of this one's group
    for (size_t g = 0; g < r->fam.size(); ++g)
      if (!perms[g].empty() && ((int)g == pg || partner[g] == (int)f || (pg >= 0 && partner[g] == pg))) done = (int)g;
    if (done >= 0) {
      const std::vector<size_t> old = idx;
      for (size_t q = 0; q < n; ++q) idx[q] = old[perms[done][q]];
      perms[f] = perms[done];
    } else {
      sort_family(r, F, idx, j.T, perms[f]);
    }
    // label prefixes: {name=" then ",name=" ; closed by "}
    j.lab.resize(nl);
    size_t fixed = F.metric.size() + 2 + (nl ? 2 : 0);  // ' ' '\n' and '"}'
    for (size_t k = 0; k < nl; ++k) {
      j.lab[k] = (k ? "\"," : "{") + F.names[F.by_name[k]] + "=\"";
      fixed += j.lab[k].size();
    }
    j.at.assign(n + 1, 0);
    std::vector<uint64_t> part(j.T + 1, 0);
    run_par(j.T, [&](unsigned t) {  // lengths, then chunk sums
      char scratch[32];
      std::vector<const char *> v(nl);
      uint64_t sum = 0;
      for (size_t q = n * t / j.T; q < n * (t + 1) / j.T; ++q) {
        const SeriesRec &sr = r->series[idx[q]];
        uint64_t len = fixed + put_value(scratch, sr.value);
        if (!sr.esc) {
          len += sr.len - nl;
        } else {
          series_values(r, sr, nl, v.data());
          for (size_t k = 0; k < nl; ++k) len += escaped_len(v[k]);
        }
        j.at[q + 1] = len;
        sum += len;
      }
      part[t + 1] = sum;
    });
    for (unsigned t = 0; t < j.T; ++t) part[t + 1] += part[t];
    run_par(j.T, [&](unsigned t) {  // offsets
      uint64_t o = part[t];
      const size_t hi = n * (t + 1) / j.T;
      for (size_t q = n * t / j.T; q < hi; ++q) {
        // the chunk's last length is not needed, and its word j.at[hi] is the next
        // chunk's first offset, which that chunk's thread writes (TSan, round 6)
        const uint64_t len = q + 1 < hi ? j.at[q + 1] : 0;
        j.at[q] = o;
        o += len;
      }
    });
    j.at[n] = part[j.T];
    j.size = part[j.T];
  }
  uint64_t N = 0;
  for (Job &j : jobs) {
    j.base = N;
    N += j.size;
  }
  if (r->text_cap < N + 1 && r->pool) {  // the pool's buffer when it is large enough
    std::lock_guard<std::mutex> lk(r->pool->mu);
    if (r->pool->text_cap >= N + 1) {
      r->text = std::move(r->pool->text);
      r->text_cap = r->pool->text_cap;
      r->pool->text_cap = 0;
    }
  }
  if (r->text_cap < N + 1) {  // (not zeroed: every byte is written below, page faults spread over the threads)
    r->text.reset(new char[N + 1]);
    r->text_cap = N + 1;
  }
  r->text_len = N;
  char *out = r->text.get();
  out[N] = '\0';
  for (Job &j : jobs) {
    if (j.text || !j.own.empty()) {
      const std::string &t = j.text ? *j.text : j.own;
      memcpy(out + j.base, t.data(), t.size());
      continue;
    }
    const ResultFamily &F = r->fam[j.f];
    const std::vector<size_t> &idx = by_fam[j.f];
    const size_t nl = F.names.size(), n = idx.size();
    run_par(j.T, [&](unsigned t) {
      std::vector<const char *> v(nl);
      const size_t q1 = n * (t + 1) / j.T;
      for (size_t q = n * t / j.T; q < q1; ++q) {
        if (q + 8 < q1) {  // the series 8 ahead: its labels are a random arena line
          const SeriesRec &ahead = r->series[idx[q + 8]];
          __builtin_prefetch(r->arenas[ahead.arena].data() + ahead.off);
        }
        const size_t i = idx[q];
        const SeriesRec &sr = r->series[i];
        char *w = out + j.base + j.at[q];
        memcpy(w, F.metric.data(), F.metric.size());
        w += F.metric.size();
        series_values(r, sr, nl, v.data());
        const char *end = r->arenas[sr.arena].data() + sr.off + sr.len;
        for (size_t k = 0; k < nl; ++k) {
          memcpy(w, j.lab[k].data(), j.lab[k].size());
          w += j.lab[k].size();
          const size_t p = F.by_name[k];
          if (!sr.esc) {
            const size_t L = (size_t)((p + 1 < nl ? v[p + 1] : end) - v[p]) - 1;
            memcpy(w, v[p], L);
            w += L;
          } else {
            w = escape_raw(w, v[p]);
          }
        }
        if (nl) {
          *w++ = '"';
          *w++ = '}';
        }
        *w++ = ' ';
        w += put_value(w, sr.value);
        *w++ = '\n';
      }
    });
  }
}
}  // namespace

int gpuagg_result_render_text(const gpuagg_result *r, char *buf, size_t cap, size_t *len) {
  if (!r || !len) return GPUAGG_EINVAL;
  std::call_once(r->text_once, [r] { render_text(r); });  // two /metrics readers may race here
  *len = r->text_len;
  if (!buf) return GPUAGG_OK;
  if (cap < r->text_len + 1) return GPUAGG_ECAPACITY;
  memcpy(buf, r->text.get(), r->text_len + 1);
  return GPUAGG_OK;
}

int gpuagg_result_text(const gpuagg_result *r, const char **text, size_t *len) {
  if (!r || !text || !len) return GPUAGG_EINVAL;
  std::call_once(r->text_once, [r] { render_text(r); });
  *text = r->text.get();
  *len = r->text_len;
  return GPUAGG_OK;
}

int gpuagg_result_series(const gpuagg_result *r, size_t i, const char **metric, uint32_t *n_labels,
                         const char *const **names, const char *const **values, uint64_t *value) {
  if (!r || i >= r->series.size()) return GPUAGG_EINVAL;
  const SeriesRec &s = r->series[i];
  const ResultFamily &f = r->fam[s.fam];
  if (metric) *metric = f.metric.c_str();
  if (n_labels) *n_labels = (uint32_t)f.names.size();
  if (names) *names = f.name_ptrs.data();
  if (values) {
    std::call_once(r->ptrs_once, [r] { build_value_ptrs(r); });
    *values = r->value_ptrs.data() + r->voff[i];
  }
  if (value) *value = s.value;
  return GPUAGG_OK;
}

void gpuagg_result_free(gpuagg_result *r) {
  if (!r) return;
  if (r->pool) {  // the large buffers back to the ctx's pool (kept: at most a few sets)
    std::lock_guard<std::mutex> lk(r->pool->mu);
    ScrapePool &p = *r->pool;
    if (p.arenas.size() < 64)
      for (auto &a : r->arenas) p.arenas.push_back(std::move(a));
    if (p.toks.size() < 64)
      for (auto &t : r->toks) p.toks.push_back(std::move(t));
    if (r->series.capacity() > p.series.capacity()) p.series.swap(r->series);
    if (r->text_cap > p.text_cap) {
      p.text = std::move(r->text);
      p.text_cap = r->text_cap;
    }
  }
  delete r;
}

// ---- sketches ---------------------------------------------------------------------
int gpuagg_sketch_refresh(gpuagg_ctx *c) {
  if (!c) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  if ((rc = fold_pending(c))) return rc;
  HIPCHK(c, x_sync(c, c->stream));
  c->h_cms.resize(c->cms_len);
  c->h_hll.resize(c->hll_len);
  if (c->cms_len) HIPCHK(c, x_copy(c, c->h_cms.data(), c->d_cms, c->cms_len * 4, hipMemcpyDeviceToHost));
  if (c->hll_len) HIPCHK(c, x_copy(c, c->h_hll.data(), c->d_hll, c->hll_len, hipMemcpyDeviceToHost));
  return GPUAGG_OK;
}

int gpuagg_cms_estimate(gpuagg_ctx *c, uint32_t src, uint32_t dst, uint32_t ports, uint32_t proto,
                        uint64_t *est) {
  if (!c || !est) return GPUAGG_EINVAL;
  if (!c->cms_len || c->h_cms.size() != c->cms_len) return fail(c, GPUAGG_ESTATE, "no count-min snapshot");
  const uint64_t base = cms_base(src, dst, ports, proto);
  const uint32_t wmask = (1u << c->cfg.cms_width_log2) - 1u;
  uint64_t m = ~0ull;
  for (uint32_t r = 0; r < c->cfg.cms_depth; ++r)
    m = std::min<uint64_t>(m, c->h_cms[((size_t)r << c->cfg.cms_width_log2) + cms_col(base, r, wmask)]);
  *est = m;
  return GPUAGG_OK;
}

int gpuagg_hll_estimate(gpuagg_ctx *c, int32_t slot, double *est) {
  if (!c || !est) return GPUAGG_EINVAL;
  if (!c->hll_len || c->h_hll.size() != c->hll_len) return fail(c, GPUAGG_ESTATE, "no HLL snapshot");
  if (slot < 0 || (uint32_t)slot >= c->key_cap) return GPUAGG_EINVAL;
  const uint32_t p = c->cfg.hll_precision;
  const size_t m = (size_t)1 << p;
  const uint8_t *reg = &c->h_hll[(size_t)slot << p];
  double sum = 0;
  size_t zeros = 0;
  for (size_t i = 0; i < m; ++i) {
    sum += std::ldexp(1.0, -(int)reg[i]);
    zeros += reg[i] == 0;
  }
  const double md = (double)m;
  const double alpha = 0.7213 / (1.0 + 1.079 / md);
  double e = alpha * md * md / sum;
  if (e <= 2.5 * md && zeros) e = md * std::log(md / (double)zeros);  // linear counting
  *est = e;
  return GPUAGG_OK;
}

int gpuagg_cms_copy(gpuagg_ctx *c, uint32_t *out, size_t n) {
  if (!c || !out || n < c->cms_len) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  if ((rc = fold_pending(c))) return rc;
  HIPCHK(c, x_sync(c, c->stream));
  if (c->cms_len) HIPCHK(c, x_copy(c, out, c->d_cms, c->cms_len * 4, hipMemcpyDeviceToHost));
  return GPUAGG_OK;
}

int gpuagg_hll_copy(gpuagg_ctx *c, uint8_t *out, size_t n) {
  if (!c || !out || n < c->hll_len) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  if ((rc = fold_pending(c))) return rc;
  HIPCHK(c, x_sync(c, c->stream));
  if (c->hll_len) HIPCHK(c, x_copy(c, out, c->d_hll, c->hll_len, hipMemcpyDeviceToHost));
  return GPUAGG_OK;
}

// ---- multi-GPU merge hooks -----------------------------------------------------------
int gpuagg_state(gpuagg_ctx *c, gpuagg_state_desc *o) {
  if (!c || !o) return GPUAGG_EINVAL;
  if (c->lat_pend.active) {  // the latency words below are read by the caller
    int rc = bind(c);
    if (rc || (rc = lat_resolve(c))) return rc;
  }
  if (c->pend.active || c->sk_pend.active) {  // the arrays below are read by the caller: fold what is waiting
    int rc = bind(c);
    if (rc || (rc = fold_pending(c))) return rc;
    HIPCHK(c, x_sync(c, c->stream));
  }
  o->dense_count = c->d_dense_cnt;
  o->dense_bytes = c->d_dense_byt;
  o->dense_len = c->dense_len;
  o->cms = c->d_cms;
  o->cms_len = c->cms_len;
  o->hll = c->d_hll;
  o->hll_len = c->hll_len;
  o->sparse_entry_words = kSparseEntryWords;
  o->sparse_len = c->sparse_slots;
  // the latency words a merge sums: both histograms (buckets, count, sum) and no_response
  // (the gaps between them are zero); the clock and the carried requests stay per shard
  o->latency = c->d_lat ? (uint64_t *)c->d_lat + kLatHist : nullptr;
  o->latency_len = c->d_lat ? kLatStateWords - kLatHist : 0;
  return GPUAGG_OK;
}

int gpuagg_sparse_export(gpuagg_ctx *c, uint64_t *dev_out, size_t cap, size_t *n_out) {
  if (!c || !n_out) return GPUAGG_EINVAL;
  *n_out = 0;
  if (!c->sparse_slots) return GPUAGG_OK;
  int rc = bind(c);
  if (rc) return rc;
  if ((rc = fold_pending(c))) return rc;
  if (c->cpu) {
    const size_t n = cpu::sparse_export(c->sv, c->sparse_slots, dev_out, cap);
    *n_out = std::min(n, cap);
    if (n > cap) return fail(c, GPUAGG_ECAPACITY, "export buffer holds %zu of %zu entries", cap, n);
    return GPUAGG_OK;
  }
  HIPCHK(c, x_set_async(c, c->d_counter, 0, 8, c->stream));
  ENQ(c);
  HIPCHK(c, launch_sparse_export(c->sv, c->sparse_slots, dev_out, cap, c->d_counter, c->stream));
  uint64_t n = 0;
  HIPCHK(c, x_copy_async(c, &n, c->d_counter, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, x_sync(c, c->stream));
  *n_out = (size_t)std::min<uint64_t>(n, cap);
  if (n > cap) return fail(c, GPUAGG_ECAPACITY, "export buffer holds %zu of %llu entries", cap, (unsigned long long)n);
  return GPUAGG_OK;
}

int gpuagg_sparse_import(gpuagg_ctx *c, const uint64_t *dev_in, size_t n) {
  if (!c || (n && !dev_in)) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  if (!n) return GPUAGG_OK;
  if ((rc = ensure_sparse(c))) return rc;
  if ((rc = fold_pending(c))) return rc;  // (CPU backend: the table has one writer at a time)
  if (c->cpu) {
    cpu::sparse_import(c->sv, dev_in, n);
    return GPUAGG_OK;
  }
  ENQ(c);
  HIPCHK(c, launch_sparse_import(c->sv, dev_in, n, c->stream));
  HIPCHK(c, x_sync(c, c->stream));
  return GPUAGG_OK;
}

int gpuagg_device_count(int *n) {
  if (!n) return GPUAGG_EINVAL;
  *n = 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) return GPUAGG_EDEVICE;
  for (int d = 0; d < ndev; ++d) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) == hipSuccess && strncmp(prop.gcnArchName, "gfx950", 6) == 0) ++*n;
  }
  return GPUAGG_OK;
}

// gpuagg_merge over RCCL (one process driving every GPU of the node): in one group, a
// reduce to ctxs[0] per state array -- dense counters, count-min and the latency words
// summed, HLL registers max-ed, in place on ctxs[0] -- and each context's exported
// group-by entries sent to ctxs[0], which inserts-and-adds them; then ctxs[1..n) reset.
// sum for counters and count-min, max for HLL; the collectives run over
// xGMI between the devices.  Bit-exact with the peer-copy merge (linear sums, exact max).
namespace {
const char *nccl_err(ncclResult_t r) { return ncclGetErrorString(r); }

int merge_rccl(gpuagg_ctx *const *ctxs, size_t n, const std::vector<int> &devs) {
  gpuagg_ctx *c0 = ctxs[0];
  int rc;
  if (c0->rccl_devs != devs) {  // communicators for this device list (created once)
    for (ncclComm_t cm : c0->rccl_comms) ncclCommDestroy(cm);
    c0->rccl_comms.assign(n, nullptr);
    c0->rccl_devs.clear();
    ncclResult_t r = ncclCommInitAll(c0->rccl_comms.data(), (int)n, devs.data());
    if (r != ncclSuccess) {
      c0->rccl_comms.clear();
      return fail(c0, GPUAGG_EDEVICE, "ncclCommInitAll(%zu devices): %s", n, nccl_err(r));
    }
    c0->rccl_devs = devs;
  }
  const std::vector<ncclComm_t> &comm = c0->rccl_comms;
  // group-by entries: exported on every context first (the counts size the transfers)
  std::vector<size_t> m(n, 0);
  size_t total = 0;
  for (size_t i = 1; i < n && c0->sparse_slots; ++i) {
    gpuagg_ctx *ci = ctxs[i];
    if ((rc = bind(ci))) return rc;
    if (ci->export_cap < ci->sparse_slots) {
      dev_free(ci, ci->d_export);
      ci->export_cap = 0;
      if ((rc = dev_alloc(ci, &ci->d_export, ci->sparse_slots * kSparseEntryWords))) return rc;
      ci->export_cap = ci->sparse_slots;
    }
    if ((rc = gpuagg_sparse_export(ci, ci->d_export, ci->export_cap, &m[i]))) return rc;
    total += m[i];
  }
  if ((rc = bind(c0))) return rc;
  uint64_t *ent = nullptr;
  if (total && (rc = dev_alloc(c0, &ent, total * kSparseEntryWords))) return rc;
  const bool lat = c0->lat_enabled != 0;
  for (size_t i = 0; i < n; ++i)
    if (lat && !ctxs[i]->d_lat) {
      dev_free(c0, ent);
      return fail(c0, GPUAGG_ESTATE, "merge: ctx %zu has no latency state", i);
    }
  ncclResult_t r = ncclGroupStart();
  size_t off = 0;
  for (size_t i = 0; i < n && r == ncclSuccess; ++i) {
    gpuagg_ctx *ci = ctxs[i];
    hipSetDevice(ci->device);
    auto reduce = [&](void *buf, size_t count, ncclDataType_t t, ncclRedOp_t op) {
      if (r == ncclSuccess && count) r = ncclReduce(buf, buf, count, t, op, 0, comm[i], ci->stream);
    };
    reduce(ci->d_dense_cnt, c0->dense_len, ncclUint64, ncclSum);
    reduce(ci->d_dense_byt, c0->dense_len, ncclUint64, ncclSum);
    reduce(ci->d_cms, c0->cms_len, ncclUint32, ncclSum);
    reduce(ci->d_hll, c0->hll_len, ncclUint8, ncclMax);
    if (lat) {
      reduce(ci->d_lat + kLatHist, kLatPeakLive - kLatHist, ncclUint64, ncclSum);
      reduce(ci->d_lat + kLatPeakLive, kLatStateWords - kLatPeakLive, ncclUint64, ncclMax);
    }
    if (i > 0 && m[i] && r == ncclSuccess)
      r = ncclSend(ci->d_export, m[i] * kSparseEntryWords, ncclUint64, 0, comm[i], ci->stream);
  }
  for (size_t i = 1; i < n && r == ncclSuccess; ++i) {
    if (!m[i]) continue;
    hipSetDevice(c0->device);
    r = ncclRecv(ent + off * kSparseEntryWords, m[i] * kSparseEntryWords, ncclUint64, (int)i, comm[0], c0->stream);
    off += m[i];
  }
  const ncclResult_t r2 = ncclGroupEnd();
  if (r == ncclSuccess) r = r2;
  for (size_t i = 0; i < n; ++i) {  // every stream idle
    hipSetDevice(ctxs[i]->device);
    hipError_t e = hipStreamSynchronize(ctxs[i]->stream);
    if (e != hipSuccess && r == ncclSuccess) {
      dev_free(c0, ent);
      return fail(c0, GPUAGG_EDEVICE, "merge: %s", hipGetErrorString(e));
    }
  }
  if (r != ncclSuccess) {
    dev_free(c0, ent);
    return fail(c0, GPUAGG_EDEVICE, "merge over RCCL: %s", nccl_err(r));
  }
  if ((rc = bind(c0))) return rc;
  rc = total ? gpuagg_sparse_import(c0, ent, total) : GPUAGG_OK;
  dev_free(c0, ent);
  if (rc) return rc;
  for (size_t i = 1; i < n; ++i)
    if ((rc = gpuagg_reset(ctxs[i]))) return rc;
  return bind(c0);
}
}  // namespace

int gpuagg_merge(gpuagg_ctx *const *ctxs, size_t n) {
  for (size_t i = 0; ctxs && i < n; ++i)
    if (ctxs[i]) ENQ(ctxs[i]);
  if (!ctxs || !n || !ctxs[0]) return GPUAGG_EINVAL;
  gpuagg_ctx *c0 = ctxs[0];
  int rc;
  const bool host = c0->cpu != nullptr;  // CPU backend: host copies and loops
  // compatibility: one metric plan and one slot / DNS dictionary on every ctx
  size_t cap = c0->key_cap;
  for (size_t i = 1; i < n; ++i) {
    const gpuagg_ctx *ci = ctxs[i];
    if (!ci || ci == c0) return fail(c0, GPUAGG_EINVAL, "merge: ctx %zu is null or the target", i);
    if ((ci->cpu != nullptr) != host)
      return fail(c0, GPUAGG_EINVAL, "merge: ctx %zu and the target are on different backends", i);
    bool same = ci->remote == c0->remote && ci->groups.size() == c0->groups.size() &&
                ci->cms_len == c0->cms_len && ci->cfg.hll_precision == c0->cfg.hll_precision &&
                (ci->sparse_slots != 0) == (c0->sparse_slots != 0) && ci->slots.size() == c0->slots.size() &&
                ci->dns.size() == c0->dns.size();
    for (size_t g = 0; same && g < c0->groups.size(); ++g)
      same = ci->groups[g].family == c0->groups[g].family && ci->groups[g].sparse == c0->groups[g].sparse &&
             ci->groups[g].src_opts == c0->groups[g].src_opts && ci->groups[g].dst_opts == c0->groups[g].dst_opts;
    for (size_t k = 0; same && k < c0->slots.size(); ++k)
      same = ci->slots[k].ns == c0->slots[k].ns && ci->slots[k].pod == c0->slots[k].pod &&
             ci->slots[k].wk_kind == c0->slots[k].wk_kind && ci->slots[k].wk_name == c0->slots[k].wk_name &&
             ci->slots[k].has_owner == c0->slots[k].has_owner && ci->slots[k].in_use == c0->slots[k].in_use;
    for (size_t k = 0; same && k < c0->dns.size(); ++k)
      same = ci->dns[k].in_use == c0->dns[k].in_use && ci->dns[k].rcode == c0->dns[k].rcode &&
             ci->dns[k].nresp == c0->dns[k].nresp &&
             ci->dns[k].qtypes == c0->dns[k].qtypes && ci->dns[k].query == c0->dns[k].query &&
             ci->dns[k].ips == c0->dns[k].ips;
    if (!same)
      return fail(c0, GPUAGG_EINVAL, "merge: ctx %zu has another metric plan or slot/DNS dictionary", i);
    cap = std::max<size_t>(cap, ci->key_cap);
  }
  // one layout everywhere (the largest slot coverage), then every stream idle
  for (size_t i = 0; i < n; ++i) {
    gpuagg_ctx *ci = ctxs[i];
    if ((rc = bind(ci))) return rc;
    if ((rc = fold_pending(ci))) return rc;
    if (ci->key_cap < cap && (rc = layout_dense(ci, (uint32_t)cap, true))) return rc;
    HIPCHK(ci, x_sync(ci, ci->stream));
    HIPCHK(ci, x_sync(ci, ci->copy_stream));
  }
  if ((rc = bind(c0))) return rc;
  // distinct devices: the RCCL collectives over xGMI (merge_rccl); contexts sharing a
  // device (several engines on one GPU) take the peer-copy path below
  if (!host) {
    std::vector<int> devs;
    for (size_t i = 0; i < n; ++i) devs.push_back(ctxs[i]->device);
    std::vector<int> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const char *mode = getenv("GPUAGG_MERGE");
    if (std::unique(sorted.begin(), sorted.end()) == sorted.end() && !(mode && !strcmp(mode, "peer")))
      return merge_rccl(ctxs, n, devs);
  }
  const size_t tmp_bytes = std::max({c0->dense_len * 8, c0->cms_len * 4, c0->hll_len, (size_t)8});
  uint8_t *tmp = nullptr;
  if ((rc = dev_alloc(c0, &tmp, tmp_bytes))) return rc;
  uint64_t *ent = nullptr;
  size_t ent_cap = 0;
  auto cleanup = [&] {
    dev_free(c0, tmp);
    dev_free(c0, ent);
  };
  auto peer = [&](void *dst, const void *src, int src_dev, size_t bytes) -> hipError_t {
    if (host) {
      memcpy(dst, src, bytes);
      return hipSuccess;
    }
    return hipMemcpyPeerAsync(dst, c0->device, src, src_dev, bytes, c0->stream);
  };
  auto add_u64 = [&](uint64_t *d, const uint64_t *x, size_t m) -> hipError_t {
    if (!host) return launch_merge_add_u64(d, x, m, c0->stream);
    for (size_t k = 0; k < m; ++k) d[k] += x[k];
    return hipSuccess;
  };
  auto add_u32 = [&](uint32_t *d, const uint32_t *x, size_t m) -> hipError_t {
    if (!host) return launch_merge_add_u32(d, x, m, c0->stream);
    for (size_t k = 0; k < m; ++k) d[k] += x[k];
    return hipSuccess;
  };
  auto max_u8 = [&](uint8_t *d, const uint8_t *x, size_t m) -> hipError_t {
    if (!host) return launch_merge_max_u8(d, x, m, c0->stream);
    for (size_t k = 0; k < m; ++k) d[k] = std::max(d[k], x[k]);
    return hipSuccess;
  };
  for (size_t i = 1; i < n; ++i) {
    gpuagg_ctx *ci = ctxs[i];
    hipError_t e = hipSuccess;
    if (c0->dense_len) {
      if ((e = peer(tmp, ci->d_dense_cnt, ci->device, c0->dense_len * 8)) == hipSuccess)
        e = add_u64(c0->d_dense_cnt, (const uint64_t *)tmp, c0->dense_len);
      if (e == hipSuccess && (e = peer(tmp, ci->d_dense_byt, ci->device, c0->dense_len * 8)) == hipSuccess)
        e = add_u64(c0->d_dense_byt, (const uint64_t *)tmp, c0->dense_len);
    }
    if (e == hipSuccess && c0->cms_len && (e = peer(tmp, ci->d_cms, ci->device, c0->cms_len * 4)) == hipSuccess)
      e = add_u32(c0->d_cms, (const uint32_t *)tmp, c0->cms_len);
    if (e == hipSuccess && c0->hll_len && (e = peer(tmp, ci->d_hll, ci->device, c0->hll_len)) == hipSuccess)
      e = max_u8(c0->d_hll, tmp, c0->hll_len);
    if (e == hipSuccess) e = x_sync(c0, c0->stream);
    if (e != hipSuccess) {
      cleanup();
      return fail(c0, GPUAGG_EDEVICE, "merge of ctx %zu: %s", i, hipGetErrorString(e));
    }
    if (ci->sparse_slots) {  // group-by entries: exported on ci, inserted-and-added on c0
      if ((rc = bind(ci))) break;
      if (ci->export_cap < ci->sparse_slots) {
        dev_free(ci, ci->d_export);
        ci->export_cap = 0;
        if ((rc = dev_alloc(ci, &ci->d_export, ci->sparse_slots * kSparseEntryWords))) break;
        ci->export_cap = ci->sparse_slots;
      }
      size_t m = 0;
      if ((rc = gpuagg_sparse_export(ci, ci->d_export, ci->export_cap, &m))) break;
      if ((rc = bind(c0))) break;
      if (m > ent_cap) {
        dev_free(c0, ent);
        ent_cap = 0;
        if ((rc = dev_alloc(c0, &ent, m * kSparseEntryWords))) break;
        ent_cap = m;
      }
      if (m) {
        if ((e = peer(ent, ci->d_export, ci->device, m * kSparseEntryWords * 8)) == hipSuccess)
          e = x_sync(c0, c0->stream);
        if (e != hipSuccess) {
          rc = fail(c0, GPUAGG_EDEVICE, "merge: %s", hipGetErrorString(e));
          break;
        }
        if ((rc = gpuagg_sparse_import(c0, ent, m))) break;
      }
    }
    if (c0->lat_enabled && ci->d_lat && c0->d_lat) {  // histograms / no_response: summed on the host
      unsigned long long a0[kLatStateWords], ai[kLatStateWords];
      if ((rc = bind(ci))) break;
      HIPCHK(ci, x_copy(ci, ai, ci->d_lat, sizeof ai, hipMemcpyDeviceToHost));
      if ((rc = bind(c0))) break;
      HIPCHK(c0, x_copy(c0, a0, c0->d_lat, sizeof a0, hipMemcpyDeviceToHost));
      for (uint32_t w = kLatHist; w < kLatStateWords; ++w) a0[w] = w < kLatPeakLive ? a0[w] + ai[w] : std::max(a0[w], ai[w]);
      HIPCHK(c0, x_copy(c0, c0->d_lat, a0, sizeof a0, hipMemcpyHostToDevice));
    }
    if ((rc = gpuagg_reset(ci))) break;
    if ((rc = bind(c0))) break;
  }
  cleanup();
  if (rc) return rc;
  HIPCHK(c0, x_sync(c0, c0->stream));
  return GPUAGG_OK;
}

int gpuagg_set_apiserver_ips(gpuagg_ctx *c, const uint32_t *ipv4, size_t n) {
  if (!c || (n && !ipv4)) return GPUAGG_EINVAL;
  if (n > kLatMaxApi) return fail(c, GPUAGG_ECAPACITY, "%zu apiserver IPs exceed %u", n, kLatMaxApi);
  int rc = bind(c);
  if (rc) return rc;
  HIPCHK(c, x_sync(c, c->stream));  // in-flight batches read the old set
  if (!c->d_api && (rc = dev_alloc(c, &c->d_api, kLatMaxApi))) return rc;
  c->api_ips.assign(ipv4, ipv4 + n);
  if (n) HIPCHK(c, x_copy(c, c->d_api, ipv4, n * 4, hipMemcpyHostToDevice));
  return GPUAGG_OK;
}

int gpuagg_ipcache_set(gpuagg_ctx *c, const uint32_t *ipv4, const uint32_t *identity, const uint32_t *meta_id,
                       size_t n) {
  if (!c || (n && (!ipv4 || !identity || !meta_id))) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  // open addressing, linear probing, load <= 50 %; the last entry for an IP wins
  size_t cap = 64;
  while (cap < 2 * n) cap <<= 1;
  const uint32_t seed = 0x7F4A7C15u, mask = (uint32_t)(cap - 1);
  std::vector<uint4> tab(cap, uint4{kIpcEmpty, 0u, 0u, 0u});
  uint32_t max_probe = 0;
  for (size_t i = 0; i < n; ++i) {
    if (ipv4[i] == kIpcEmpty) return fail(c, GPUAGG_ERANGE, "255.255.255.255 cannot be an ipcache key");
    uint32_t h = ip_h1(ipv4[i], seed) & mask, p = 0;
    while (tab[h].x != kIpcEmpty && tab[h].x != ipv4[i]) {
      h = (h + 1) & mask;
      ++p;
    }
    tab[h] = uint4{ipv4[i], identity[i], meta_id[i], 0u};
    max_probe = std::max(max_probe, p);
  }
  HIPCHK(c, x_sync(c, c->stream));  // in-flight decodes read the old image
  if (cap != c->ipc_cap) {
    dev_free(c, c->d_ipc);
    c->ipc_cap = 0;
    if ((rc = dev_alloc(c, &c->d_ipc, cap))) return rc;
    c->ipc_cap = cap;
  }
  HIPCHK(c, x_copy(c, c->d_ipc, tab.data(), cap * sizeof(uint4), hipMemcpyHostToDevice));
  c->ipc_seed = seed;
  c->ipc_max_probe = max_probe;
  return GPUAGG_OK;
}

int gpuagg_hubble_decode_device(gpuagg_ctx *c, const gpuagg_columns *in, size_t n, const gpuagg_hubble_cols *out) {
  if (!c || !in || !out) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  if (n == 0) return GPUAGG_OK;
  if (!in->src_ip || !in->dst_ip || !in->meta || !out->src_identity || !out->dst_identity || !out->src_meta ||
      !out->dst_meta || !out->summary_kind || !out->summary_arg)
    return fail(c, GPUAGG_EINVAL, "hubble decode: null column");
  if (!c->ipc_cap) {  // no image yet: every IP resolves to World
    if ((rc = gpuagg_ipcache_set(c, nullptr, nullptr, nullptr, 0))) return rc;
  }
  HubbleArgs a{};
  a.table = c->d_ipc;
  a.mask = (uint32_t)(c->ipc_cap - 1);
  a.seed = c->ipc_seed;
  a.max_probe = c->ipc_max_probe;
  a.src = in->src_ip;
  a.dst = in->dst_ip;
  a.meta = in->meta;
  a.dns = in->dns_id;
  a.n = n;
  a.o_sid = out->src_identity;
  a.o_did = out->dst_identity;
  a.o_smeta = out->src_meta;
  a.o_dmeta = out->dst_meta;
  a.o_kind = out->summary_kind;
  a.o_arg = out->summary_arg;
  if (c->cpu) c->cpu->hubble(a);
  else {
    ENQ(c);
    HIPCHK(c, launch_hubble(a, c->n_cu, c->stream));
  }
  return GPUAGG_OK;
}

int gpuagg_enrich_device(gpuagg_ctx *c, const gpuagg_columns *in, size_t n, int32_t *src_slot,
                         int32_t *dst_slot) {
  if (!c || !in) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  if (n == 0) return GPUAGG_OK;
  if (!in->src_ip || !in->dst_ip || !src_slot || !dst_slot)
    return fail(c, GPUAGG_EINVAL, "enrich: null column");
  if (!c->ip_cap) return fail(c, GPUAGG_ESTATE, "gpuagg_set_endpoints was never called");
  return enrich_launch(c, in->src_ip, in->dst_ip, n, src_slot, dst_slot);
}

int gpuagg_set_time_offset(gpuagg_ctx *c, int64_t ns) {
  if (!c) return GPUAGG_EINVAL;
  c->time_offset = ns;
  return GPUAGG_OK;
}

int gpuagg_latency_read(gpuagg_ctx *c, gpuagg_latency_state *out) {
  if (!c || !out) return GPUAGG_EINVAL;
  int rc = bind(c);
  if (rc) return rc;
  *out = gpuagg_latency_state{};
  out->enabled = c->lat_enabled;
  if (!c->d_lat) return GPUAGG_OK;
  if ((rc = lat_resolve(c))) return rc;
  unsigned long long w[kLatStateWords];
  HIPCHK(c, x_sync(c, c->stream));
  HIPCHK(c, x_copy(c, w, c->d_lat, sizeof w, hipMemcpyDeviceToHost));
  for (int i = 0; i < 11; ++i) {
    out->latency_buckets[i] = w[kLatHist + i];
    out->handshake_buckets[i] = w[kLatHandshake + i];
  }
  out->latency_count = w[kLatHist + 11];
  out->latency_sum = (int64_t)w[kLatHist + 12];
  out->handshake_count = w[kLatHandshake + 11];
  out->handshake_sum = (int64_t)w[kLatHandshake + 12];
  out->no_response = w[kLatNoResponse];
  out->pending = w[kLatPending];
  out->peak_pending = std::max<uint64_t>(c->lat_peak_pending, w[kLatPending]);
  out->peak_live = w[kLatPeakLive];
  out->capacity_evictions = w[kLatCapEvictions];
  out->capacity_batches = w[kLatCapBatches];
  out->limit = c->cfg.latency_limit ? c->cfg.latency_limit : kLatLimit;
  return GPUAGG_OK;
}

int gpuagg_get_stats(gpuagg_ctx *c, gpuagg_stats *out) {
  if (!c || !out) return GPUAGG_EINVAL;
  if (!c->cpu) {
    if (int rc = bind(c)) return rc;
    drain_timing(c);  // the timed launches since the last read (their events complete by now or soon)
  }
  *out = c->stats;
  return GPUAGG_OK;
}

int gpuagg_set_timing(gpuagg_ctx *c, int enabled) {
  if (!c) return GPUAGG_EINVAL;
  if (!c->cpu) {  // events of launches before this call count before it
    if (int rc = bind(c)) return rc;
    drain_timing(c);
  }
  if (c->cpu) c->host_timing = enabled != 0;  // host wall time of the launches (no HIP events)
  else c->timing = enabled != 0;
  c->tm_chain = false;
  if (!enabled) {  // the timed counters start again from zero
    c->stats.kernel_ms = 0;
    c->stats.fold_ms = 0;
    c->stats.kernel_launches = 0;
    c->stats.sketch_ms = 0;
    c->stats.sketch_launches = 0;
    c->stats.decode_ms = 0;
    c->stats.decode_launches = 0;
  }
  return GPUAGG_OK;
}

void *gpuagg_stream(gpuagg_ctx *c) { return c && !c->cpu ? (void *)c->stream : nullptr; }

const char *gpuagg_build_id(void) { return GPUAGG_BUILD_ID; }

}  // extern "C"

namespace {
// Splits [0, n) over host threads for the standalone shard functions (one thread below
// 2^18 records: thread start-up would cost more than the hashing).
template <class F>
void shard_threads(size_t n, F &&f) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const unsigned T = n < (1u << 18) ? 1u : std::min(16u, hw);
  if (T == 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 1; t < T; ++t) th.emplace_back([&, t] { f(n * t / T, n * (t + 1) / T); });
  f(0, n / T);
  for (auto &x : th) x.join();
}
}  // namespace

extern "C" {

// dist.shard_of (shard_5tuple): the device of each record.
int gpuagg_shard_columns(const uint32_t *src, const uint32_t *dst, const uint32_t *ports, const uint32_t *meta,
                         size_t n, uint32_t n_shards, uint32_t *out) {
  if (!n) return GPUAGG_OK;
  if (!src || !dst || !meta || !out || !n_shards) return GPUAGG_EINVAL;
  shard_threads(n, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) out[i] = shard_5tuple(src[i], dst[i], ports ? ports[i] : 0u, meta[i], n_shards);
  });
  return GPUAGG_OK;
}

int gpuagg_shard_raw(int kind, const void *raw, size_t n, uint32_t n_shards, uint32_t *out) {
  if (!n) return GPUAGG_OK;
  if (!raw || !out || !n_shards || (kind != GPUAGG_RAW_PACKET && kind != GPUAGG_RAW_DROP)) return GPUAGG_EINVAL;
  auto u32 = [](const uint8_t *q) { uint32_t v; memcpy(&v, q, 4); return v; };
  // field offsets: conntrack.c:34-49 (src 12, dst 16, ports 20, proto 42) and
  // drop_reason.c:39-54 (src 0, dst 4, ports 8, proto 22); ports as HostToNetShort decodes them
  const size_t sz = kind == GPUAGG_RAW_PACKET ? GPUAGG_RAW_PACKET_SIZE : GPUAGG_RAW_DROP_SIZE;
  const size_t o_ip = kind == GPUAGG_RAW_PACKET ? 12 : 0, o_port = o_ip + 8;
  const size_t o_proto = kind == GPUAGG_RAW_PACKET ? 42 : 22;
  shard_threads(n, [&](size_t lo, size_t hi) {
    const uint8_t *p = (const uint8_t *)raw + lo * sz;
    for (size_t i = lo; i < hi; ++i, p += sz)
      out[i] = shard_5tuple(u32(p + o_ip), u32(p + o_ip + 4), raw_swap_ports(u32(p + o_port)), p[o_proto], n_shards);
  });
  return GPUAGG_OK;
}

const char *gpuagg_kernel_name(const gpuagg_ctx *c) { return c ? c->kernel_name.c_str() : ""; }
const char *gpuagg_sketch_kernel_name(const gpuagg_ctx *c) { return c ? c->sketch_kernel_name.c_str() : ""; }

}  // extern "C"
