// CPU backend of the flow-aggregation engine (GPUAGG_FLAG_CPU_BACKEND): the same plan,
// state layout and ABI as the gfx950 kernels, executed by host threads on host memory,
// for nodes without a usable GPU (SURVEY.md 8b "A CPU backend behind the same ABI"; the
// reference runs its loop on every node's CPU, metrics_module.go:276-317).
//
// New product code, not the oracle: it restates the kernels' per-record semantics
// (gpuagg_kernels.hip apply_groups / sparse_add / sketch_update, gpuagg_decode.hip,
// gpuagg_hubble.hip, gpuagg_latency.hip), so the runtime's host side -- registry, slots,
// IP cache, dictionaries, snapshot rendering, export -- works unchanged on its state:
//   * dense counters: per-thread private arrays, summed into the ctx's arrays by flush()
//     (the runtime calls it wherever the GPU path folds deferred lists);
//   * group-by keys: per-thread hash maps of (k0, k1, k2) -> (count, bytes), inserted
//     into the ctx's table (same 5-word / compact layout and probe sequence) by flush();
//   * sketches: relaxed atomics on the shared count-min rows / HLL registers;
//   * latency: the TTL join run sequentially in record order (the GPU's per-key walk
//     gives the same result; gpuagg_latency.hip).
#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <deque>
#include <unordered_map>
#include <vector>

#include "gpuagg_internal.h"
#include "gpuagg_launch.h"

namespace gpuagg {
namespace cpu {

namespace {

struct Lk {
  int32_t slot;
  uint32_t api;
};

Lk lk_from(uint64_t e) {
  if (e == kIpEmpty) return Lk{-1, 0};
  return Lk{(int32_t)((e >> 32) & ((1u << kSlotBits) - 1)), (uint32_t)(e >> 53) & 1u};
}

// The HBM IP table's lookup (ip_lookup in gpuagg_kernels.hip): radix blocks when the
// runtime built them, else the 2-choice bucket table.
struct IpTable {
  const uint64_t *slots;
  uint32_t mask, seed;
  const uint16_t *pre;
  const uint32_t *blk;
  Lk lookup(uint32_t ip) const {
    if (pre) {
      const uint32_t b = pre[ip & 0xFFFFu];
      if (b == kRadixNoBlock) return Lk{-1, 0};
      const uint32_t e = blk[((size_t)b << 16) | (ip >> 16)];
      return e == kRadixEmpty ? Lk{-1, 0} : Lk{(int32_t)(e & ((1u << kSlotBits) - 1)), e >> 31};
    }
    for (uint32_t b : {ip_h1(ip, seed) & mask, ip_h2(ip, seed) & mask})
      for (int k = 0; k < 2; ++k) {
        const uint64_t e = slots[2 * (size_t)b + k];
        if (e != kIpEmpty && (uint32_t)e == ip) return lk_from(e);
      }
    return Lk{-1, 0};
  }
};

struct Key {
  uint64_t k0, k1, k2;
  bool operator==(const Key &o) const { return k0 == o.k0 && k1 == o.k1 && k2 == o.k2; }
};
struct KeyHash {
  size_t operator()(const Key &k) const { return (size_t)key_hash(k.k0, k.k1, k.k2); }
};
using KeyMap = std::unordered_map<Key, std::pair<uint64_t, uint64_t>, KeyHash>;

uint32_t side_port17(uint8_t opts, uint32_t port, uint32_t proto) {
  return ((opts & OPT_PORT) && (proto == 6 || proto == 17)) ? (0x10000u | port) : 0u;
}

// One record through every group (apply_groups of gpuagg_kernels.hip, one lane).
template <class D, class S>
void apply_groups(const Plan &p, D &&dense, S &&sparse, uint32_t sip, uint32_t dip, uint32_t nbytes, uint32_t meta,
                  uint32_t ports, uint32_t dns, const Lk &ls, const Lk &ld) {
  const uint32_t proto = meta_proto(meta), verdict = meta_verdict(meta);
  const uint32_t tdir = meta_tdir(meta), reason = meta_reason(meta), dnstype = meta_dnstype(meta);
  const uint32_t flagmask = (verdict == kVerdictForwarded && proto == 6) ? flag_label_mask(meta_flags(meta)) : 0u;
  const uint32_t sport = ports & 0xFFFFu, dport = ports >> 16;
  auto hit_of = [&](uint32_t fam) {
    switch (fam) {
      case FAM_FWD: return verdict == kVerdictForwarded;
      case FAM_DROP: return verdict == kVerdictDropped;
      case FAM_TCPFLAGS: return verdict == kVerdictForwarded && proto == 6 && flagmask != 0;
      case FAM_RETRANS: return verdict == kVerdictRetrans;
      case FAM_DNS_REQ: return verdict == kVerdictDns && dnstype == kDnsQuery;
      case FAM_DNS_RESP: return verdict == kVerdictDns && dnstype == kDnsResponse;
    }
    return false;
  };
  struct SideKey {
    uint32_t ip, slot1, port17;
  };
  auto side_key = [&](uint8_t opts, uint32_t ip, const Lk &lk, uint32_t port) {
    return SideKey{(opts & OPT_IP) ? ip : 0u, (opts & OPT_EP) ? (uint32_t)(lk.slot + 1) : 0u,
                   side_port17(opts, port, proto)};
  };
  for (int g = 0; g < p.ngroups; ++g) {
    const GroupPlan &gp = p.g[g];
    const uint32_t fam = gp.family;
    if (!hit_of(fam)) continue;
    const uint32_t addb = fam <= FAM_DROP ? nbytes : 0u;
    if (p.local) {
      if (gp.src_opts == 0) continue;  // getLocalCtxValues (types.go:379-416)
      const bool s_ok = ls.slot >= 0 && !ls.api, d_ok = ld.slot >= 0 && !ld.api;
      if (fam == FAM_DNS_REQ || fam == FAM_DNS_RESP) {  // dns.go:506-540: one update
        if (!s_ok && !d_ok) continue;
        const int side = (s_ok && d_ok) ? (tdir == 1 ? 0 : 1) : (d_ok ? 0 : 1);
        const SideKey k = side == 0 ? side_key(gp.src_opts, dip, ld, dport) : side_key(gp.src_opts, sip, ls, sport);
        sparse(key0(g, (uint32_t)side, k.slot1, k.ip), key1(k.port17, 0, 0), key2(0, dns), 0u);
        continue;
      }
      for (int side = 0; side < 2; ++side) {  // 0 ingress (dst), 1 egress (src)
        if (!(side == 0 ? d_ok : s_ok)) continue;
        const Lk &lk = side == 0 ? ld : ls;
        if (!gp.sparse) {
          const uint32_t key = gp.key_mode ? (uint32_t)lk.slot : 0u;
          const uint64_t row = gp.dense_base + ((uint64_t)key * 2u + (uint32_t)side) * gp.nsub;
          if (fam == FAM_TCPFLAGS) {
            for (uint32_t m = flagmask; m; m &= m - 1) dense(row + __builtin_ctz(m), 0u);
          } else {
            dense(row + (fam == FAM_DROP ? reason : 0u), addb);
          }
          continue;
        }
        const SideKey k = side == 0 ? side_key(gp.src_opts, dip, ld, dport) : side_key(gp.src_opts, sip, ls, sport);
        if (fam == FAM_TCPFLAGS) {
          for (uint32_t m = flagmask; m; m &= m - 1)
            sparse(key0(g, ((uint32_t)__builtin_ctz(m) << 3) | (uint32_t)side, k.slot1, k.ip), key1(k.port17, 0, 0),
                   0ull, 0u);
        } else {
          const uint32_t sub = ((fam == FAM_DROP ? reason : 0u) << 3) | (uint32_t)side;
          sparse(key0(g, sub, k.slot1, k.ip), key1(k.port17, 0, 0), 0ull, addb);
        }
      }
      continue;
    }
    // remote context: one tuple [prefix labels] + source values + destination values
    const SideKey ks = side_key(gp.src_opts, sip, ls, sport), kd = side_key(gp.dst_opts, dip, ld, dport);
    const uint64_t k1 = key1(ks.port17, kd.port17, kd.slot1);
    if (fam == FAM_TCPFLAGS) {
      for (uint32_t m = flagmask; m; m &= m - 1)
        sparse(key0(g, (uint32_t)__builtin_ctz(m) << 3, ks.slot1, ks.ip), k1, key2(kd.ip, 0), 0u);
      continue;
    }
    uint32_t sub = 0, dnsv = 0;
    if (fam == FAM_FWD || fam == FAM_RETRANS) sub = tdir << 1;
    else if (fam == FAM_DROP) sub = (reason << 3) | (tdir << 1);
    else dnsv = dns;
    sparse(key0(g, sub, ks.slot1, ks.ip), k1, key2(kd.ip, dnsv), addb);
  }
}

// sparse_add / sparse_add_compact of gpuagg_kernels.hip on host memory (one writer:
// flush() runs single-threaded).
void table_add(const SparseView &s, uint64_t k0, uint64_t k1, uint64_t k2, uint64_t c, uint64_t b) {
  if (s.compact) {
    const uint64_t key = k0 | (k2 & 0xFFFFFFFFULL);
    const uint32_t h = (uint32_t)fmix64(key ^ 0x243F6A8885A308D3ULL) & s.mask;
    const uint32_t smask = (1u << s.seg_log2) - 1u, seg = h & ~smask;
    for (uint32_t probe = 0; probe <= smask; ++probe) {
      uint64_t *slot = s.k0 + 2ull * (seg | ((h + probe) & smask));
      if (slot[0] == 0 || slot[0] == key) {
        slot[0] = key;
        slot[1] += c;
        return;
      }
    }
    *s.dropped += c;
    return;
  }
  const uint32_t h0 = (uint32_t)key_hash(k0, k1, k2) & s.mask, smask = (1u << s.seg_log2) - 1u;
  const uint32_t seg = h0 & ~smask, nprobe = smask < kSparseMaxProbe ? smask + 1u : kSparseMaxProbe;
  for (uint32_t probe = 0; probe < nprobe; ++probe) {
    uint64_t *w = s.k0 + (size_t)(seg | ((h0 + probe) & smask)) * kSparseSlotWords;
    if (w[0] == 0) {
      w[0] = k0;
      w[1] = k1;
      w[2] = k2;
      w[3] = c;
      w[4] = b;
      return;
    }
    if (w[0] == k0 && w[1] == k1 && w[2] == k2) {
      w[3] += c;
      w[4] += b;
      return;
    }
  }
  *s.dropped += c;
}

// Splits [0, n) over the engine's threads.
template <class F>
void parallel(unsigned threads, size_t n, F &&f) {
  const unsigned t = (unsigned)std::max<size_t>(1, std::min<size_t>(threads, (n + 4095) / 4096));
  if (t <= 1) {
    f(0u, (size_t)0, n);
    return;
  }
  std::vector<std::thread> pool;
  const size_t per = (n + t - 1) / t;
  for (unsigned i = 0; i < t; ++i) {
    const size_t lo = std::min(n, i * per), hi = std::min(n, lo + per);
    pool.emplace_back([&f, i, lo, hi] { f(i, lo, hi); });
  }
  for (auto &th : pool) th.join();
}

}  // namespace

// Per-thread accumulators between flushes.
struct Engine::Part {
  std::vector<uint64_t> cnt, byt;
  KeyMap keys;
};

Engine::Engine(unsigned threads) : threads_(threads ? threads : 1) {}
Engine::~Engine() = default;

void Engine::aggregate(const LaunchArgs &a) {
  if (!a.n) return;
  const bool sparse_on = a.sparse.k0 != nullptr;
  if (parts_.size() < threads_) parts_.resize(threads_);
  for (auto &p : parts_)
    if (!p) p.reset(new Part());
  const IpTable t{a.ip_slots, a.ip_mask, a.ip_seed, a.ip_pre, a.ip_blk};
  dense_len_ = a.dense_len;
  dense_cnt_ = a.dense_cnt;
  dense_byt_ = a.dense_byt;
  sparse_ = a.sparse;
  parallel(threads_, a.n, [&](unsigned ti, size_t lo, size_t hi) {
    Part &P = *parts_[ti];
    if (P.cnt.size() < a.dense_len) {
      P.cnt.resize(a.dense_len, 0);
      P.byt.resize(a.dense_len, 0);
    }
    auto dense = [&](uint64_t bin, uint32_t nb) {
      P.cnt[bin] += 1;
      P.byt[bin] += nb;
    };
    auto sparse = [&](uint64_t k0, uint64_t k1, uint64_t k2, uint32_t nb) {
      if (!sparse_on) return;
      auto &v = P.keys[Key{k0, k1, k2}];
      v.first += 1;
      v.second += nb;
    };
    const ColsView &c = a.cols;
    for (size_t i = lo; i < hi; ++i) {
      const uint32_t s = c.src_ip[i], d = c.dst_ip[i];
      apply_groups(a.plan, dense, sparse, s, d, c.bytes ? c.bytes[i] : 0u, c.meta[i], c.ports ? c.ports[i] : 0u,
                   c.dns_id ? c.dns_id[i] : 0u, t.lookup(s), t.lookup(d));
    }
  });
  pending_ = true;
}

void Engine::flush() {
  if (!pending_) return;
  pending_ = false;
  for (auto &pp : parts_) {
    if (!pp) continue;
    Part &P = *pp;
    const size_t nb = std::min<size_t>(P.cnt.size(), dense_len_);
    for (size_t i = 0; i < nb; ++i) {
      if (P.cnt[i]) {
        dense_cnt_[i] += P.cnt[i];
        dense_byt_[i] += P.byt[i];
      }
    }
    std::fill(P.cnt.begin(), P.cnt.end(), 0);
    std::fill(P.byt.begin(), P.byt.end(), 0);
    for (const auto &kv : P.keys) table_add(sparse_, kv.first.k0, kv.first.k1, kv.first.k2, kv.second.first,
                                            kv.second.second);
    P.keys.clear();
  }
}

void Engine::drop() {
  pending_ = false;
  for (auto &pp : parts_) {
    if (!pp) continue;
    std::fill(pp->cnt.begin(), pp->cnt.end(), 0);
    std::fill(pp->byt.begin(), pp->byt.end(), 0);
    pp->keys.clear();
  }
}

// sketch_update of gpuagg_kernels.hip: count-min +1 per row, HLL register max.
void Engine::sketch(const SketchArgs &s) {
  const IpTable t{s.ip_slots, s.ip_mask, s.ip_seed, s.ip_pre, s.ip_blk};
  const uint32_t wmask = (1u << s.cms_wlog2) - 1u;
  parallel(threads_, s.n, [&](unsigned, size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      const uint32_t src = s.cols.src_ip[i], dst = s.cols.dst_ip[i];
      if (s.cms_depth) {
        const uint64_t base = cms_base(src, dst, s.cols.ports ? s.cols.ports[i] : 0u, meta_proto(s.cols.meta[i]));
        for (uint32_t r = 0; r < s.cms_depth; ++r)
          __atomic_fetch_add(&s.cms[((size_t)r << s.cms_wlog2) + cms_col(base, r, wmask)], 1u, __ATOMIC_RELAXED);
      }
      if (s.hll_p) {
        const Lk ls = t.lookup(src);
        if (ls.slot < 0 || (uint32_t)ls.slot >= s.hll_slots) continue;
        const uint64_t h = hll_hash(dst);
        const uint32_t idx = (uint32_t)(h >> (64 - s.hll_p));
        const uint8_t rho = (uint8_t)(__builtin_clzll((h << s.hll_p) | (1ULL << (s.hll_p - 1))) + 1);
        uint8_t *r = s.hll + ((size_t)ls.slot << s.hll_p) + idx;
        uint8_t old = __atomic_load_n(r, __ATOMIC_RELAXED);
        while (old < rho && !__atomic_compare_exchange_n(r, &old, rho, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
        }
      }
    }
  });
}

// packet_decode_kernel / drop_decode_kernel of gpuagg_decode.hip.
uint64_t Engine::decode(const DecodeArgs &a) {
  std::atomic<uint64_t> bad{0};
  const OutCols &o = a.out;
  parallel(threads_, a.n, [&](unsigned, size_t lo, size_t hi) {
    uint64_t nbad = 0;
    for (size_t i = lo; i < hi; ++i) {
      uint32_t w[18];
      const bool pkt = a.kind == kRawPacket;
      memcpy(w, (const uint8_t *)a.raw + i * (pkt ? 72 : 32), pkt ? 72 : 32);
      const RawRow r = pkt ? decode_packet_words(w, a.time_offset) : decode_drop_words(w, a.time_offset);
      nbad += r.bad;
      o.src_ip[i] = r.src;
      o.dst_ip[i] = r.dst;
      o.bytes[i] = r.bytes;
      o.meta[i] = r.meta;
      if (o.ports) o.ports[i] = r.ports;
      if (o.dns_id) o.dns_id[i] = 0xFFFFFFFFu;
      if (o.tcp_id) o.tcp_id[i] = r.tcp_id;
      if (o.time_ns) o.time_ns[i] = r.time_ns;
    }
    bad += nbad;
  });
  return bad.load();
}

// enrich_kernel of gpuagg_kernels.hip.
void Engine::enrich(const EnrichArgs &a) {
  const IpTable t{a.ip_slots, a.ip_mask, a.ip_seed, a.ip_pre, a.ip_blk};
  parallel(threads_, a.n, [&](unsigned, size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      a.o_src[i] = t.lookup(a.src[i]).slot;
      a.o_dst[i] = t.lookup(a.dst[i]).slot;
    }
  });
}

// hubble_decode_kernel of gpuagg_hubble.hip.
void Engine::hubble(const HubbleArgs &a) {
  auto look = [&](uint32_t ip, uint32_t &id, uint32_t &meta) {
    id = kIdentityWorld;
    meta = kIpcNoMeta;
    if (!a.table) return;
    uint32_t h = ip_h1(ip, a.seed) & a.mask;
    for (uint32_t p = 0; p <= a.max_probe; ++p, h = (h + 1) & a.mask) {
      const uint4 e = a.table[h];
      if (e.x == ip) {
        id = e.y;
        meta = e.z;
        return;
      }
      if (e.x == kIpcEmpty) return;
    }
  };
  parallel(threads_, a.n, [&](unsigned, size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      look(a.src[i], a.o_sid[i], a.o_smeta[i]);
      look(a.dst[i], a.o_did[i], a.o_dmeta[i]);
      const uint32_t m = a.meta[i], proto = meta_proto(m), verdict = meta_verdict(m);
      uint32_t kind = kSummaryNone, arg = 0;
      if (verdict == kVerdictDns) {
        kind = kSummaryDns;
        arg = (a.dns ? a.dns[i] & 0x3FFFFFFFu : 0u) | (meta_dnstype(m) << 30);
      } else if (verdict == kVerdictDropped) {
        kind = kSummaryDrop;
        arg = meta_reason(m);
      } else if (proto == 6) {
        if (verdict == kVerdictForwarded || verdict == kVerdictRetrans) {
          kind = kSummaryTcp;
          arg = meta_flags(m);
        }
      } else if (proto == 17) {
        kind = kSummaryUdp;
      }
      a.o_kind[i] = kind;
      a.o_arg[i] = arg;
    }
  });
}

// The TTL join of gpuagg_latency.hip in record order, as the ttlcache runs it: before each
// latency event the items whose expiry the clock has passed are evicted (no_response);
// a request inserts unless its key is live, in which case the Get hit touches it
// (expiry = clock + TTL, front of the LRU list); a Set with `limit` live items first
// evicts the least recently touched one (uncounted); a reply observes and deletes.  At
// the batch end items past the end clock expire and the rest carry over in LRU order.
// The clock of a row is the running maximum of the record times.
void Engine::latency(const LatArgs &a, uint32_t enabled) {
  unsigned long long *st = a.state;
  struct E {
    uint64_t expires, seq;
    uint32_t nanos;
    bool syn;
  };
  std::unordered_map<Key, E, KeyHash> live;
  std::deque<std::pair<uint64_t, Key>> lru;  // (touch seq, key), stale once the key is touched again
  const uint64_t limit = a.limit ? a.limit : kLatLimit;
  for (const auto &c : carry_) {  // carried in LRU order
    live[Key{c.k0, c.k1, 0}] = E{c.clock, c.seq, c.nanos, ((c.bits >> 2) & 1u) != 0};
    lru.emplace_back(c.seq, Key{c.k0, c.k1, 0});
  }
  carry_.clear();
  // the least recently touched live item (stale records dropped), or live.end()
  auto front = [&]() {
    while (!lru.empty()) {
      auto it = live.find(lru.front().second);
      if (it != live.end() && it->second.seq == lru.front().first) return it;
      lru.pop_front();
    }
    return live.end();
  };
  auto is_api = [&](uint32_t ip) {
    for (uint32_t i = 0; i < a.n_api; ++i)
      if (a.api[i] == ip) return true;
    return false;
  };
  auto bucket = [](int64_t v) -> uint32_t { return v <= 0 ? 0u : v >= 5 ? 10u : (uint32_t)(2 * v); };
  uint64_t clk = st[kLatClock];
  uint64_t seq = st[kLatSeqBase], peak = live.size();
  bool bound = false;  // the capacity evicted in this batch (the device's sequential-pass batches)
  for (size_t i = 0; i < a.n; ++i) {
    clk = std::max<uint64_t>(clk, a.time_ns[i]);
    const uint32_t m = a.meta[i];
    if ((m & 0xFFu) != 6u || a.tcp_id[i] == 0u) continue;
    const uint32_t obs = m >> 30;
    const uint32_t role = obs == 3u ? 1u : obs == 2u ? 2u : 0u;
    if (!role || !(is_api(a.src[i]) || is_api(a.dst[i]))) continue;
    const uint64_t my_seq = seq++;
    for (auto f = front(); f != live.end() && clk > f->second.expires; f = front()) {
      live.erase(f);  // evicted by the cleaner before this record
      lru.pop_front();
      if (enabled & 4u) st[kLatNoResponse] += 1;
    }
    const uint32_t s = a.src[i], d = a.dst[i], p = a.ports[i], sp = p & 0xFFFFu, dp = p >> 16;
    const uint64_t id = a.tcp_id[i];
    const uint64_t k0 = role == 1u ? ((uint64_t)s | ((uint64_t)d << 32)) : ((uint64_t)d | ((uint64_t)s << 32));
    const uint64_t k1 = role == 1u ? ((uint64_t)sp | ((uint64_t)dp << 16) | (id << 32))
                                   : ((uint64_t)dp | ((uint64_t)sp << 16) | (id << 32));
    const uint32_t verdict = (m >> 8) & 0xFFu, flags = (m >> 21) & 0x3Fu;
    const bool has_flags = verdict == kVerdictForwarded || verdict == kVerdictRetrans;
    const bool syn = has_flags && (flags & 2u), ack = has_flags && (flags & 16u);
    const uint32_t nanos = (uint32_t)(a.time_ns[i] % 1000000000ULL);
    const Key key{k0, k1, 0};
    auto it = live.find(key);
    if (role == 1u) {
      if (it != live.end()) {  // Get hit: touched
        it->second.expires = clk + kLatTtlNs;
        it->second.seq = my_seq;
      } else {
        if (live.size() >= limit) {  // Set at capacity: the LRU back goes, uncounted
          live.erase(front());
          lru.pop_front();
          st[kLatCapEvictions] += 1;
          bound = true;
        }
        live[key] = E{clk + kLatTtlNs, my_seq, nanos, syn};
        peak = std::max<uint64_t>(peak, live.size());
      }
      lru.emplace_back(my_seq, key);
    } else if (it != live.end()) {
      const int64_t dd = (int64_t)nanos - (int64_t)it->second.nanos, ad = dd < 0 ? -dd : dd;
      const int64_t lat = (dd < 0 ? -1 : 1) * ((ad + 500000) / 1000000);  // math.Round
      const uint32_t bk = bucket(lat);
      if (enabled & 1u) {
        st[kLatHist + bk] += 1;
        st[kLatHist + 11] += 1;
        st[kLatHist + 12] += (unsigned long long)lat;
      }
      if ((enabled & 2u) && it->second.syn && syn && ack) {
        st[kLatHandshake + bk] += 1;
        st[kLatHandshake + 11] += 1;
        st[kLatHandshake + 12] += (unsigned long long)lat;
      }
      live.erase(it);
    }
  }
  for (auto f = front(); f != live.end(); f = front()) {  // batch end, LRU order
    if (clk > f->second.expires) {
      if (enabled & 4u) st[kLatNoResponse] += 1;
    } else {
      carry_.push_back(LatEvent{f->first.k0, f->first.k1, f->second.expires, f->second.seq, f->second.nanos,
                                3u | (f->second.syn ? 4u : 0u)});
    }
    live.erase(f);
    lru.pop_front();
  }
  st[kLatSeqBase] = seq;
  st[kLatClock] = clk;
  st[kLatPending] = carry_.size();
  st[kLatPeakLive] = std::max<uint64_t>(st[kLatPeakLive], peak);
  st[kLatCapBatches] += bound ? 1u : 0u;
}

void Engine::latency_reset() { carry_.clear(); }

// ---- table maintenance (sparse_init / export / import kernels) ----------------------------
void sparse_init(const SparseView &v, size_t slots) {
  if (v.compact) {
    memset(v.k0, 0, slots * 16);
    return;
  }
  for (size_t i = 0; i < slots; ++i) {
    uint64_t *w = v.k0 + i * kSparseSlotWords;
    w[0] = w[1] = w[3] = w[4] = 0;
    w[2] = kKeyPending;
  }
}

size_t sparse_export(const SparseView &v, size_t slots, uint64_t *out, size_t cap) {
  size_t n = 0;
  for (size_t i = 0; i < slots; ++i) {
    uint64_t e[kSparseEntryWords];
    if (v.compact) {
      const uint64_t key = v.k0[2 * i];
      if (!key) continue;
      e[0] = key & 0xFFFFFFFF00000000ULL;
      e[1] = 0;
      e[2] = key & 0xFFFFFFFFULL;
      e[3] = v.k0[2 * i + 1];
      e[4] = 0;
    } else {
      const uint64_t *w = v.k0 + i * kSparseSlotWords;
      if (!w[0]) continue;
      for (int k = 0; k < kSparseEntryWords; ++k) e[k] = w[k];
    }
    if (n < cap) memcpy(out + n * kSparseEntryWords, e, sizeof e);
    ++n;
  }
  return n;
}

void sparse_import(const SparseView &v, const uint64_t *in, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const uint64_t *e = in + i * kSparseEntryWords;
    table_add(v, e[0], e[1], e[2], e[3], e[4]);
  }
}

void zero_slots(uint64_t *cnt, uint64_t *byt, uint8_t *hll, uint32_t hll_p, const uint32_t *dead, uint32_t ndead,
                const Plan &p) {
  for (uint32_t k = 0; k < ndead; ++k) {
    const uint32_t slot = dead[k];
    if (cnt)
      for (int g = 0; g < p.ngroups; ++g) {
        const GroupPlan &gp = p.g[g];
        if (gp.sparse || !gp.key_mode) continue;
        const uint64_t lo = gp.dense_base + (uint64_t)slot * 2u * gp.nsub;
        for (uint32_t i = 0; i < 2u * gp.nsub; ++i) cnt[lo + i] = byt[lo + i] = 0;
      }
    if (hll) memset(hll + ((size_t)slot << hll_p), 0, (size_t)1 << hll_p);
  }
}

}  // namespace cpu
}  // namespace gpuagg
