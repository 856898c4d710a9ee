// Node-wide ingestion feeds (include/gpuagg.h gpuagg_raw_feed_*): the hand-over of the
// packetparser / dropreason reader loop (packetparser_linux.go:556-654, whose two decode
// workers run processRecord per perf sample, :669-696) and of the Go plugin's decoded
// record slices, to one engine context per device.
//
// Per device the feed keeps TWO pinned host stagings of `capacity` records: while the H2D
// DMA of a full one runs (submitted without waiting for it, gx_submit_*_async), the other
// fills, and a staging is only refilled after its own copy-done event.  Each put is split
// over a small pool of host threads:
//   * one device: every thread copies / decodes a contiguous range of the records straight
//     to its position (the range may straddle the two stagings);
//   * several devices: pass 1, every thread computes the device of each record of its range
//     (shard_5tuple, the function of dist.shard_of) and counts them per device; the
//     per-device prefix over the threads gives every thread its write positions, so pass 2
//     scatters in input order -- each device receives exactly the records gpuagg_shard_raw
//     assigns it, in order.
// Raw samples are either copied as they are and decoded on the GPU (the default,
// GPUAGG_FEED_RAW_DMA: packet_decode_kernel / drop_decode_kernel; the host does one memcpy
// per sample, so the agent's CPU cost stays lowest) or decoded on the host threads into
// pinned SoA columns (GPUAGG_FEED_HOST_DECODE: only the columns the metric plan reads cross
// PCIe -- 16 B per record for forward/drop instead of the 72-byte sample -- for ~4x the host
// work per sample).  Both produce the same columns (decode_packet_words /
// decode_drop_words restate the kernels).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "gpuagg_feed.h"
#include "gpuagg_internal.h"

using namespace gpuagg;

namespace {

constexpr unsigned kMaxFeedThreads = 64;
// Default host threads: one device is PCIe-bound at 4 (raw samples at ~54 GB/s, 7.6e8
// records/s on MI355X; more threads only contend with the DMA for host memory), several
// devices have a link each and take more (host_fed_raw).
constexpr unsigned kDefaultThreadsOne = 4, kDefaultThreadsMany = 16;

// A persistent pool: run(f) calls f(t) for t = 0..n-1, t = 0 on the caller, and returns
// when all have finished.  Workers spin for a short while after a job (back-to-back puts
// dispatch in ~1 us), then sleep on a condition variable (an idle feed costs nothing).
class Pool {
 public:
  explicit Pool(unsigned n) : n_(n) {
    for (unsigned i = 1; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_.store(true, std::memory_order_relaxed);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  unsigned size() const { return n_; }

  template <class F>
  void run(F &&f) {
    if (n_ == 1) {
      f(0u);
      return;
    }
    // feeds share pools (shared_pool): one job at a time (uncontended under the ABI's
    // one-thread-per-ctx rule, since the plugin's feeds span the same contexts)
    std::lock_guard<std::mutex> job(run_mu_);
    fn_ = [](void *p, unsigned t) { (*static_cast<F *>(p))(t); };
    arg_ = &f;
    left_.store(n_ - 1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(m_);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    f(0u);
    while (left_.load(std::memory_order_acquire)) __builtin_ia32_pause();
  }

 private:
  static constexpr int kSpin = 1 << 14;  // ~50-100 us of pause before sleeping
  void loop(unsigned i) {
    uint64_t seen = 0;
    for (;;) {
      uint64_t g = gen_.load(std::memory_order_acquire);
      for (int s = 0; g == seen && s < kSpin; ++s) {
        __builtin_ia32_pause();
        g = gen_.load(std::memory_order_acquire);
      }
      if (g == seen) {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
        g = gen_.load(std::memory_order_acquire);
      }
      seen = g;
      if (stop_.load(std::memory_order_relaxed)) return;
      fn_(arg_, i);
      left_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  const unsigned n_;
  std::vector<std::thread> th_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<unsigned> left_{0};
  std::atomic<bool> stop_{false};
  std::mutex m_, run_mu_;
  std::condition_variable cv_;
  void (*fn_)(void *, unsigned) = nullptr;
  void *arg_ = nullptr;
};

// One pool per thread count for the whole process: the Go plugin's packet, drop and record
// feeds (and any feeds of other plugins) share one set of host threads instead of starting
// up to 16 spinning threads each.  The last feed that lets go of a pool joins it.
std::shared_ptr<Pool> shared_pool(unsigned n) {
  static std::mutex mu;
  static std::map<unsigned, std::weak_ptr<Pool>> pools;
  std::lock_guard<std::mutex> g(mu);
  std::shared_ptr<Pool> p = pools[n].lock();
  if (!p) {
    p = std::make_shared<Pool>(n);
    pools[n] = p;
  }
  return p;
}

inline void split(size_t n, unsigned parts, unsigned t, size_t &lo, size_t &hi) {
  lo = n * t / parts;
  hi = n * (t + 1) / parts;
}

inline uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

// Rows a thread buffers per device before writing them to a staging.  Pinned host memory
// takes scattered 4-byte stores badly (each column is a separate stream of partial
// lines): rows are decoded / transposed into this cache-resident tile and written out
// with one contiguous copy per column, like the raw samples' straight memcpy.
constexpr size_t kTileRows = 1024;
struct Tile {
  size_t n = 0;      // rows buffered
  uint64_t bad = 0;  // out-of-range rows decoded into this tile since the put began
  uint32_t col[7][kTileRows];  // src, dst, bytes, meta, ports, dns_id, tcp_id
  uint64_t time_ns[kTileRows];
  uint8_t raw[kTileRows * GPUAGG_RAW_PACKET_SIZE];  // GPUAGG_FEED_RAW_DMA: samples as they came
};

}  // namespace

struct gpuagg_raw_feed {
  struct Stage {
    uint8_t *raw = nullptr;       // GPUAGG_FEED_RAW_DMA: capacity samples as they came
    gpuagg_batch *bat = nullptr;  // host decode / GPUAGG_RECORD: pinned SoA columns
    hipEvent_t done = nullptr;    // its H2D copies completed (device contexts)
    bool pending = false;         // submitted; `done` not yet waited for
  };
  struct Dev {
    gpuagg_ctx *c = nullptr;
    Stage st[2];
    int cur = 0;       // the staging being filled
    size_t fill = 0;   // records in it
    uint64_t submitted = 0;
    bool gone = false;  // the context was destroyed (gpuagg_destroy detached the feed)
  };
  int kind = 0;
  int mode = GPUAGG_FEED_RAW_DMA;
  bool dry = false;  // GPUAGG_FEED_DRY_RUN: stagings counted, never submitted (diagnostics)
  size_t rec = 0, cap = 0;  // bytes per input record, records per staging
  std::vector<Dev> dev;
  std::shared_ptr<Pool> pool;
  std::vector<uint16_t> shard;  // device of each record of a piece (several devices)
  std::vector<size_t> cnt;      // [thread][device]: records, then write positions
  std::vector<std::unique_ptr<Tile>> tiles;  // [thread][device]
  bool dead = false;

  bool soa() const { return kind == GPUAGG_RECORD || mode == GPUAGG_FEED_HOST_DECODE; }
  unsigned threads() const { return pool ? pool->size() : 1u; }
};

namespace {

using Feed = gpuagg_raw_feed;

int stage_wait(Feed::Dev &D, Feed::Stage &s) {
  if (!s.pending) return GPUAGG_OK;
  s.pending = false;
  if (int rc = gx_bind(D.c)) return rc;
  const hipError_t e = hipEventSynchronize(s.done);
  if (e != hipSuccess) return gx_fail(D.c, GPUAGG_EDEVICE, hipGetErrorString(e));
  return GPUAGG_OK;
}

void stage_free(Feed *f, Feed::Dev &D, Feed::Stage &s) {
  stage_wait(D, s);
  if (s.bat) gpuagg_free_batch(D.c, s.bat);
  if (s.raw) gx_host_free(D.c, s.raw);
  if (s.done) hipEventDestroy(s.done);
  s = Feed::Stage{};
  (void)f;
}

int stage_alloc(Feed *f, Feed::Dev &D, Feed::Stage &s) {
  gpuagg_ctx *c = D.c;
  if (int rc = gx_bind(c)) return rc;
  if (f->soa()) {
    if (int rc = gpuagg_alloc_batch(c, f->cap, &s.bat)) return rc;
    if (f->kind != GPUAGG_RECORD)  // raw samples carry no DNS payload: written once
      std::fill(s.bat->cols.dns_id, s.bat->cols.dns_id + f->cap, 0xFFFFFFFFu);
  } else if (gx_host_alloc(c, (void **)&s.raw, f->cap * f->rec) != GPUAGG_OK) {
    return gx_fail(c, GPUAGG_ENOMEM, "raw feed staging");
  }
  if (!gx_is_cpu(c)) {
    const hipError_t e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (e != hipSuccess) return gx_fail(c, GPUAGG_EDEVICE, hipGetErrorString(e));
  }
  return gx_prepare(c, f->cap);
}

int alloc_all(Feed *f) {
  for (auto &D : f->dev)
    for (auto &s : D.st)
      if (int rc = stage_alloc(f, D, s)) return rc;
  return GPUAGG_OK;
}

void free_all(Feed *f) {
  for (auto &D : f->dev)
    if (!D.gone)
      for (auto &s : D.st) stage_free(f, D, s);
}

void set_threads(Feed *f, unsigned t) {
  t = std::max(1u, std::min(t, kMaxFeedThreads));
  if (!f->pool || f->pool->size() != t) f->pool = shared_pool(t);
  f->cnt.assign((size_t)t * f->dev.size(), 0);
  f->tiles.resize((size_t)t * f->dev.size());
  for (auto &p : f->tiles)
    if (!p) p.reset(new Tile());
}

// Submits the first n records of device d's current staging and moves to the other one.
int submit_stage(Feed *f, Feed::Dev &D, size_t n) {
  Feed::Stage &s = D.st[D.cur];
  D.cur ^= 1;
  if (!n) return GPUAGG_OK;
  if (f->dry) {
    D.submitted += n;
    return GPUAGG_OK;
  }
  const int rc = f->soa() ? gx_submit_batch_async(D.c, s.bat, n, s.done)
                          : gx_submit_raw_async(D.c, f->kind, s.raw, n, s.done);
  if (rc == GPUAGG_OK) D.submitted += n;
  // even when the launch failed, the H2D copies out of this staging may be enqueued (and
  // s.done recorded behind them): it is not refilled or freed before that event
  s.pending = !gx_is_cpu(D.c);
  return rc;
}

// One input record appended to a thread's tile.
inline void append_row(const Feed *f, Tile &t, const uint8_t *p, uint64_t toff) {
  const size_t i = t.n++;
  if (!f->soa()) {
    memcpy(t.raw + i * f->rec, p, f->rec);
    return;
  }
  if (f->kind == GPUAGG_RECORD) {
    gpuagg_record r;
    memcpy(&r, p, sizeof r);
    t.col[0][i] = r.src_ip;
    t.col[1][i] = r.dst_ip;
    t.col[2][i] = r.bytes;
    t.col[3][i] = r.meta;
    t.col[4][i] = r.ports;
    t.col[5][i] = r.dns_id;
    t.col[6][i] = r.tcp_id;
    t.time_ns[i] = r.time_ns;
    return;
  }
  uint32_t w[GPUAGG_RAW_PACKET_SIZE / 4];
  memcpy(w, p, f->rec);
  const RawRow r = f->kind == GPUAGG_RAW_PACKET ? decode_packet_words(w, toff) : decode_drop_words(w, toff);
  t.bad += r.bad;
  t.col[0][i] = r.src;
  t.col[1][i] = r.dst;
  t.col[2][i] = r.bytes;
  t.col[3][i] = r.meta;
  t.col[4][i] = r.ports;
  t.col[6][i] = r.tcp_id;
  t.time_ns[i] = r.time_ns;
}

// Rows [a, a + k) of a tile to positions [q, q + k) of one staging.
inline void copy_rows(const Feed *f, const Tile &t, size_t a, size_t k, Feed::Stage &s, size_t q) {
  if (!f->soa()) {
    memcpy(s.raw + q * f->rec, t.raw + a * f->rec, k * f->rec);
    return;
  }
  gpuagg_columns &o = s.bat->cols;
  uint32_t *dst[7] = {o.src_ip, o.dst_ip, o.bytes, o.meta, o.ports, o.dns_id, o.tcp_id};
  for (int c = 0; c < 7; ++c)
    if (c != 5 || f->kind == GPUAGG_RECORD)  // raw samples: the dns_id column is constant
      memcpy(dst[c] + q, t.col[c] + a, k * 4);
  memcpy(o.time_ns + q, t.time_ns + a, k * 8);
}

// A device's tile to its write position `pos` (advanced), across the two stagings.
inline void flush_tile(const Feed *f, Feed::Dev &D, Tile &t, size_t &pos) {
  const size_t cap = f->cap, n = t.n;
  const size_t in_a = pos < cap ? std::min(n, cap - pos) : 0;
  if (in_a) copy_rows(f, t, 0, in_a, D.st[D.cur], pos);
  if (in_a < n) copy_rows(f, t, in_a, n - in_a, D.st[D.cur ^ 1], pos + in_a - cap);
  pos += n;
  t.n = 0;
}

// The device of one input record (gpuagg_shard_raw / gpuagg_shard_columns' function).
inline uint32_t device_of(const Feed *f, const uint8_t *p, uint32_t nd) {
  if (f->kind == GPUAGG_RECORD) {
    gpuagg_record r;
    memcpy(&r, p, sizeof r);
    return shard_5tuple(r.src_ip, r.dst_ip, r.ports, r.meta, nd);
  }
  // conntrack.c:34-49 (src 12, dst 16, ports 20, proto 42); drop_reason.c:39-54 (0, 4, 8, 22)
  const bool pkt = f->kind == GPUAGG_RAW_PACKET;
  const size_t o_ip = pkt ? 12 : 0;
  return shard_5tuple(rd32(p + o_ip), rd32(p + o_ip + 4), raw_swap_ports(rd32(p + o_ip + 8)), p[pkt ? 42 : 22], nd);
}

// One piece of m <= cap records.
int put_piece(Feed *f, const uint8_t *p, size_t m) {
  const size_t nd = f->dev.size(), rec = f->rec, cap = f->cap;
  const unsigned T = f->threads();
  std::vector<uint64_t> toff(nd);
  for (size_t d = 0; d < nd; ++d) toff[d] = gx_time_offset(f->dev[d].c);
  for (auto &tl : f->tiles) tl->bad = 0;
  std::vector<size_t> tot(nd, 0);
  if (nd == 1) {
    tot[0] = m;
  } else {
    if (f->shard.size() < m) f->shard.resize(m);
    f->pool->run([&](unsigned t) {
      size_t lo, hi;
      split(m, T, t, lo, hi);
      std::vector<size_t> cnt(nd, 0);  // thread-local: the shared array is written once
      uint16_t *sh = f->shard.data();
      for (size_t i = lo; i < hi; ++i) {
        const uint32_t d = device_of(f, p + i * rec, (uint32_t)nd);
        sh[i] = (uint16_t)d;
        ++cnt[d];
      }
      std::copy(cnt.begin(), cnt.end(), f->cnt.begin() + (size_t)t * nd);
    });
    for (size_t d = 0; d < nd; ++d) {  // counts -> each thread's first write position
      size_t pos = f->dev[d].fill;
      for (unsigned t = 0; t < T; ++t) {
        const size_t k = f->cnt[(size_t)t * nd + d];
        f->cnt[(size_t)t * nd + d] = pos;
        pos += k;
      }
      tot[d] = pos - f->dev[d].fill;
    }
  }
  // the staging being filled, and the other one where this piece runs past the end,
  // must be free of their previous DMA
  for (size_t d = 0; d < nd; ++d) {
    Feed::Dev &D = f->dev[d];
    if (int rc = stage_wait(D, D.st[D.cur])) return rc;
    if (D.fill + tot[d] > cap)
      if (int rc = stage_wait(D, D.st[D.cur ^ 1])) return rc;
  }
  f->pool->run([&](unsigned t) {
    size_t lo, hi;
    split(m, T, t, lo, hi);
    if (nd == 1 && !f->soa()) {  // straight copies, split where the range leaves the first staging
      Feed::Dev &D = f->dev[0];
      Feed::Stage &a = D.st[D.cur], &b = D.st[D.cur ^ 1];
      const size_t p0 = D.fill + lo, p1 = D.fill + hi;
      const size_t a1 = std::min(p1, cap);
      if (p0 < a1) memcpy(a.raw + p0 * rec, p + lo * rec, (a1 - p0) * rec);
      const size_t b0 = std::max(p0, cap);
      if (b0 < p1) memcpy(b.raw + (b0 - cap) * rec, p + (lo + b0 - p0) * rec, (p1 - b0) * rec);
      return;
    }
    // write positions, thread-local (one device: this thread's rows are contiguous)
    std::vector<size_t> pos(nd);
    if (nd == 1) pos[0] = f->dev[0].fill + lo;
    else std::copy(f->cnt.begin() + (size_t)t * nd, f->cnt.begin() + (size_t)(t + 1) * nd, pos.begin());
    std::unique_ptr<Tile> *tl = &f->tiles[(size_t)t * nd];
    for (size_t i = lo; i < hi; ++i) {
      const uint32_t d = nd == 1 ? 0u : f->shard[i];
      Tile &tile = *tl[d];
      append_row(f, tile, p + i * rec, toff[d]);
      if (tile.n == kTileRows) flush_tile(f, f->dev[d], tile, pos[d]);
    }
    for (size_t d = 0; d < nd; ++d)
      if (tl[d]->n) flush_tile(f, f->dev[d], *tl[d], pos[d]);
  });
  int err = GPUAGG_OK;
  for (size_t d = 0; d < nd; ++d) {
    Feed::Dev &D = f->dev[d];
    if (f->kind != GPUAGG_RECORD && f->soa()) {
      uint64_t b = 0;
      for (unsigned t = 0; t < T; ++t) b += f->tiles[(size_t)t * nd + d]->bad;
      gx_count_host_decode(D.c, tot[d], b);
    }
    D.fill += tot[d];
    if (D.fill >= cap) {  // full: its DMA starts now, the other staging holds the rest
      D.fill -= cap;
      if (int rc = submit_stage(f, D, cap)) err = err ? err : rc;
    }
  }
  return err;
}

}  // namespace

namespace gpuagg {
void feed_on_ctx_destroy(gpuagg_raw_feed *f, gpuagg_ctx *c) {
  for (auto &D : f->dev)
    if (D.c == c && !D.gone) {
      for (auto &s : D.st) stage_free(f, D, s);
      D.gone = true;
      f->dead = true;
    }
}
}  // namespace gpuagg

extern "C" {

int gpuagg_raw_feed_create(gpuagg_ctx *const *ctxs, size_t n_ctx, int kind, size_t capacity,
                           gpuagg_raw_feed **out) {
  if (!ctxs || !n_ctx || n_ctx > 65535 || !out || !capacity ||
      (kind != GPUAGG_RAW_PACKET && kind != GPUAGG_RAW_DROP && kind != GPUAGG_RECORD))
    return GPUAGG_EINVAL;
  *out = nullptr;
  for (size_t d = 0; d < n_ctx; ++d)
    if (!ctxs[d]) return GPUAGG_EINVAL;
  auto *f = new gpuagg_raw_feed();
  f->kind = kind;
  f->rec = kind == GPUAGG_RAW_PACKET ? GPUAGG_RAW_PACKET_SIZE
           : kind == GPUAGG_RAW_DROP ? GPUAGG_RAW_DROP_SIZE
                                     : sizeof(gpuagg_record);
  f->cap = capacity;
  f->dev.resize(n_ctx);
  for (size_t d = 0; d < n_ctx; ++d) {
    f->dev[d].c = ctxs[d];
    gx_feed_attach(ctxs[d], f);
  }
  set_threads(f, std::min(n_ctx == 1 ? kDefaultThreadsOne : kDefaultThreadsMany,
                          std::max(1u, std::thread::hardware_concurrency())));
  if (int rc = alloc_all(f)) {
    gpuagg_raw_feed_destroy(f);
    return rc;
  }
  *out = f;
  return GPUAGG_OK;
}

int gpuagg_raw_feed_configure(gpuagg_raw_feed *f, uint32_t threads, int mode) {
  const bool dry = mode & GPUAGG_FEED_DRY_RUN;
  mode &= ~GPUAGG_FEED_DRY_RUN;
  if (!f || (mode != GPUAGG_FEED_HOST_DECODE && mode != GPUAGG_FEED_RAW_DMA)) return GPUAGG_EINVAL;
  if (f->dead) return GPUAGG_ESTATE;
  for (auto &D : f->dev)
    if (D.fill) return gx_fail(D.c, GPUAGG_ESTATE, "gpuagg_raw_feed_configure: flush the feed first");
  if (threads) set_threads(f, threads);
  f->dry = dry;
  if (f->kind != GPUAGG_RECORD && mode != f->mode) {
    free_all(f);
    f->mode = mode;
    if (int rc = alloc_all(f)) {
      f->dead = true;  // partial stagings: later puts / flushes return GPUAGG_ESTATE
      return rc;
    }
  }
  return GPUAGG_OK;
}

int gpuagg_raw_feed_put(gpuagg_raw_feed *f, const void *raw, size_t n) {
  if (!f || (n && !raw)) return GPUAGG_EINVAL;
  if (f->dead) return GPUAGG_ESTATE;
  const uint8_t *p = (const uint8_t *)raw;
  int err = GPUAGG_OK;
  while (n) {
    const size_t m = std::min(n, f->cap);
    if (int rc = put_piece(f, p, m)) err = err ? err : rc;
    p += m * f->rec;
    n -= m;
  }
  return err;
}

int gpuagg_raw_feed_flush(gpuagg_raw_feed *f) {
  if (!f) return GPUAGG_EINVAL;
  if (f->dead) return GPUAGG_ESTATE;
  int err = GPUAGG_OK;
  for (auto &D : f->dev) {
    const size_t n = D.fill;
    D.fill = 0;
    if (n)
      if (int rc = submit_stage(f, D, n)) err = err ? err : rc;
  }
  return err;
}

int gpuagg_raw_feed_submitted(const gpuagg_raw_feed *f, uint64_t *per_ctx, size_t n_ctx) {
  if (!f || !per_ctx || n_ctx < f->dev.size()) return GPUAGG_EINVAL;
  for (size_t d = 0; d < f->dev.size(); ++d) per_ctx[d] = f->dev[d].submitted;
  return GPUAGG_OK;
}

void gpuagg_raw_feed_destroy(gpuagg_raw_feed *f) {
  if (!f) return;
  free_all(f);
  for (auto &D : f->dev)
    if (!D.gone) gx_feed_detach(D.c, f);
  delete f;
}

}  // extern "C"
