// Internal interface between the runtime (gpuagg_runtime.cpp, which owns struct
// gpuagg_ctx) and the node-wide ingestion feeds (gpuagg_feed.cpp).  Not part of the ABI.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "gpuagg.h"

namespace gpuagg {

bool gx_is_cpu(const gpuagg_ctx *c);
int gx_bind(gpuagg_ctx *c);
int gx_fail(gpuagg_ctx *c, int code, const char *msg);
// pinned host memory (device contexts) / plain host memory (CPU backend)
int gx_host_alloc(gpuagg_ctx *c, void **p, size_t n);
void gx_host_free(gpuagg_ctx *c, void *p);
// sizes the context's device staging for `cap` records (no-op on the CPU backend)
int gx_prepare(gpuagg_ctx *c, size_t cap);
uint64_t gx_time_offset(const gpuagg_ctx *c);
// Host-fed submits that return as soon as the H2D copies are ENQUEUED: `host_done` is
// recorded on the copy stream behind them, and the host buffer may be refilled once it
// has completed.  CPU-backend contexts consume the buffer before returning (host_done
// unused).  The aggregation runs async as for gpuagg_submit(_raw).
int gx_submit_batch_async(gpuagg_ctx *c, gpuagg_batch *b, size_t n, hipEvent_t host_done);
int gx_submit_raw_async(gpuagg_ctx *c, int kind, const void *host_raw, size_t n, hipEvent_t host_done);
// rows a feed decoded on the host: gpuagg_stats.decoded / decode_out_of_range
void gx_count_host_decode(gpuagg_ctx *c, uint64_t n, uint64_t out_of_range);
// the context keeps the feeds that reference it, so gpuagg_destroy can detach them
void gx_feed_attach(gpuagg_ctx *c, gpuagg_raw_feed *f);
void gx_feed_detach(gpuagg_ctx *c, gpuagg_raw_feed *f);

// gpuagg_feed.cpp: the context is being destroyed; the feed releases what it holds of it
// (its pinned stagings) and refuses further puts.
void feed_on_ctx_destroy(gpuagg_raw_feed *f, gpuagg_ctx *c);

}  // namespace gpuagg
