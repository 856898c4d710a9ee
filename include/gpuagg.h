/*
 * gpuagg.h -- C ABI of the MI355X flow-aggregation engine for Retina.
 *
 * This is the drop-in boundary that replaces the per-event Go loops of
 * matmerr/retina's enricher and advanced-metrics module (reference @ 2025-03-28):
 *
 *   Enricher.Write / Run / enrich        pkg/enricher/enricher.go:68-140,185-187
 *   Cache.GetObjByIP (snapshot)          pkg/controllers/cache/cache.go:110-169
 *   Module.Reconcile / updateMetricsContexts  pkg/module/metrics/metrics_module.go:205-264
 *   Module.run -> metric.ProcessFlow     pkg/module/metrics/metrics_module.go:276-305
 *   {Forward,DropCount,TCP,TCPRetrans,DNS}Metrics.ProcessFlow
 *                                        pkg/module/metrics/{forward,drops,tcpflags,
 *                                        tcpretrans,dns}.go
 *   GaugeVec/CounterVec.WithLabelValues  pkg/metrics/interfaces.go:12-20 (the sink)
 *
 * The caller is the Go cgo plugin in go/pkg/gpuagg, which keeps
 * the registry.Plugin interface (pkg/plugin/registry/registry.go:16-34) and feeds the
 * decoded records of packetparser / dropreason / dns / tcpretrans as column batches.
 *
 * Conventions: plain C types only; every entry returns 0 (GPUAGG_OK) or a negative
 * GPUAGG_E* code and never aborts; gpuagg_last_error() gives the message.  One ctx is
 * used by one thread at a time; every entry re-binds the ctx's HIP device, so cgo's
 * OS-thread migration is harmless.
 */
#ifndef GPUAGG_H
#define GPUAGG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPUAGG_ABI_VERSION 3u  /* 2: columns tcp_id/time_ns, stats, state latency words;
                                   3: gpuagg_config.wide_list_mib, latency_limit */

/* error codes */
#define GPUAGG_OK 0
#define GPUAGG_EINVAL (-1)     /* bad argument / spec                           */
#define GPUAGG_ENOMEM (-2)     /* host or device allocation failed               */
#define GPUAGG_EDEVICE (-3)    /* HIP runtime error or no usable gfx950 device   */
#define GPUAGG_ECAPACITY (-4)  /* a fixed-capacity table overflowed              */
#define GPUAGG_ESTATE (-5)     /* call not valid in the ctx's current state      */
#define GPUAGG_EDUPLICATE (-6) /* two metrics would register the same family     */
#define GPUAGG_ERANGE (-7)     /* value outside the encodable range              */
#define GPUAGG_ENOTFOUND (-8)  /* no such object (cache.go's "not found in cache") */

typedef struct gpuagg_ctx gpuagg_ctx;

/* ------------------------------------------------------------------------------
 * Configuration
 * ---------------------------------------------------------------------------- */
typedef struct gpuagg_config {
  uint32_t abi_version;          /* = GPUAGG_ABI_VERSION                             */
  int32_t device;                /* HIP device ordinal                               */
  int32_t remote_context;        /* cfg.RemoteContext (pkg/config/config.go:72):
                                    0 = local context, 1 = remote context            */
  uint32_t max_slots;            /* endpoint identity slots (pods), <= 2^21-2        */
  uint32_t max_ips;              /* pod IPs in the IP table                          */
  uint32_t sparse_capacity_log2; /* group-by hash table entries = 2^this (0: 22)     */
  uint32_t cms_depth;            /* count-min rows (0 = sketches off)                */
  uint32_t cms_width_log2;       /* count-min columns = 2^this                       */
  uint32_t hll_precision;        /* HyperLogLog p (registers 2^p per source pod; 0=off) */
  uint32_t flags;                /* GPUAGG_FLAG_* (0 = defaults)                     */
  uint32_t wide_list_mib;        /* device memory for the 192-bit-key segment lists of
                                    this ctx, MiB (0: min(32 GiB, device memory / 8));
                                    a full list falls back to exact memory-side atomics */
  uint32_t latency_limit;        /* node-apiserver latency: live pending requests kept,
                                    ttlcache.WithCapacity (latency.go:35,120-121);
                                    0 = the reference's LIMIT, 100000                 */
} gpuagg_config;

/* gpuagg_config.flags */
#define GPUAGG_FLAG_NO_LDS_IP_TABLE 1u /* keep the IP table in HBM/L2 only (diagnostics) */
#define GPUAGG_FLAG_DIRECT_SKETCH 2u   /* sketch updates as global atomics, no window lists (diagnostics) */
#define GPUAGG_FLAG_NO_RADIX_IP_TABLE 4u /* HBM lookups through the bucket hash table only (diagnostics) */
#define GPUAGG_FLAG_NO_HOT_KEYS 16u    /* no LDS hot-key cache in front of the group-by table (diagnostics) */
#define GPUAGG_FLAG_FOLD_PER_BATCH 8u  /* fold the spill / segment lists after every batch instead of
                                          once per gpuagg_sync or state read (diagnostics) */
#define GPUAGG_FLAG_LDS_CUCKOO 64u     /* tier-1 LDS IP image as the cuckoo table even when the radix
                                          image fits (diagnostics) */
#define GPUAGG_FLAG_ROW_RADIX 256u     /* LDS IP images in the radix form with its row table even
                                        when the dense form would do (diagnostics / tests) */
#define GPUAGG_FLAG_CPU_BACKEND 128u  /* run on host threads and host memory, no device (nodes without
                                          a gfx950 GPU): the same plan, ABI and results; "device"
                                          pointers of this ctx's calls are host pointers          */
#define GPUAGG_FLAG_NO_WIDE_LISTS 32u  /* 192-bit group-by keys straight into the table with memory-side
                                          atomics, not through per-segment lists (diagnostics) */
#define GPUAGG_FLAG_NARROW_ENTRIES 512u /* 24-byte segment-list entries instead of 32 when the plan's keys
                                          have no port / DNS fields: measured C1 -3 %, C4 remote +6 %
                                          per step (the entries are written as partial sectors)   */

int gpuagg_create(const gpuagg_config *cfg, gpuagg_ctx **out);
/* Number of gfx950 devices visible to this process (one ctx per device). */
int gpuagg_device_count(int *n);
void gpuagg_destroy(gpuagg_ctx *ctx);
const char *gpuagg_last_error(const gpuagg_ctx *ctx);

/* ------------------------------------------------------------------------------
 * Module.Reconcile: one entry per crd MetricsContextOptions
 * (crd/api/v1alpha1/metricsconfiguration_types.go:27-58).  A *_set flag of 0 means
 * the Go slice was nil (which changes behaviour, basemetricsobject.go:31-49).
 * Resets all accumulated state, like Clean() + ResetAdvancedMetricsRegistry()
 * (metrics_module.go:208-213) -- unless the options equal the current ones under
 * validations.MetricsContextOptionsCompare (same metric names, label lists equal as sets;
 * validate_metricconfiguration.go:118-160, utils/common.go:58-84), in which case Module.Reconcile
 * leaves the metrics alone (metrics_module.go:142-166) and so does this call.
 * ---------------------------------------------------------------------------- */
typedef struct gpuagg_metric_options {
  const char *metric_name;
  const char *const *source_labels;
  uint32_t n_source_labels;
  int32_t source_labels_set;
  const char *const *destination_labels;
  uint32_t n_destination_labels;
  int32_t destination_labels_set;
} gpuagg_metric_options;

int gpuagg_reconcile(gpuagg_ctx *ctx, const gpuagg_metric_options *opts, size_t n);

/* ------------------------------------------------------------------------------
 * Endpoint identity (the enricher's view of the IP cache).
 *
 * gpuagg_slot_intern returns a stable slot id for the label identity of a pod
 * (namespace, pod name, first owner reference) -- the fields getEndpoint /
 * getWorkloads copy into flow.Endpoint (enricher.go:142-183).  workload_kind ==
 * NULL means the pod has no owner references.  Slot ids are never reused within a
 * reconcile epoch, so counters keyed by slot stay valid across table swaps.
 *
 * gpuagg_set_endpoints replaces the IP -> slot map (a versioned snapshot of
 * Cache.ipToEpKey/epMap, cache.go:17-46,204-233; services and nodes resolve to no
 * endpoint, enricher.go:157-160, so they are simply absent).  It takes effect for
 * batches submitted after the call.  ipv4 values use the record encoding below.
 * ---------------------------------------------------------------------------- */
int gpuagg_slot_intern(gpuagg_ctx *ctx, const char *namespace_, const char *pod_name,
                       const char *workload_kind, const char *workload_name, int32_t *slot);
int gpuagg_set_endpoints(gpuagg_ctx *ctx, const uint32_t *ipv4, const int32_t *slot, size_t n,
                         uint64_t version);

/* ------------------------------------------------------------------------------
 * The IP cache itself (pkg/controllers/cache/cache.go), kept natively so the IP -> pod
 * map follows the reference's update/delete rules exactly: an update first deletes
 * every object holding one of its IPs -- the WHOLE object, all its IPs (deleteByIP,
 * cache.go:394-420; deleteEndpoint :315-337) -- and an IP no longer listed by an
 * updated pod keeps pointing at it (updateEndpoint :204-233).  Services and nodes own
 * IPs too (updateSvc :244-270, updateNode :282-305) and resolve to no endpoint.
 * Endpoints are keyed "namespace/name" (BaseObject.Key, baseobject.go:19-21), nodes by
 * name.  gpuagg_cache_commit installs the cache's current IP -> pod map (as
 * gpuagg_set_endpoints does) for batches submitted after it.
 * ---------------------------------------------------------------------------- */
int gpuagg_cache_update_endpoint(gpuagg_ctx *ctx, const char *namespace_, const char *pod_name,
                                 const char *workload_kind, const char *workload_name,
                                 const uint32_t *ipv4, size_t n_ips);
int gpuagg_cache_delete_endpoint(gpuagg_ctx *ctx, const char *namespace_, const char *pod_name);
int gpuagg_cache_update_service(gpuagg_ctx *ctx, const char *namespace_, const char *name, uint32_t ipv4);
int gpuagg_cache_delete_service(gpuagg_ctx *ctx, const char *namespace_, const char *name);
int gpuagg_cache_update_node(gpuagg_ctx *ctx, const char *name, uint32_t ipv4);
int gpuagg_cache_delete_node(gpuagg_ctx *ctx, const char *name);
int gpuagg_cache_commit(gpuagg_ctx *ctx, uint64_t version);

/* Slot lifecycle.  Dense counters and HLL registers are sized by the slots in use (grown
 * when an endpoint table references a new slot, up to max_slots).  gpuagg_retire_slots
 * frees every slot the installed IP table no longer references: its counters, HLL
 * registers and group-by entries are cleared and the id is reused by a later
 * gpuagg_slot_intern.  Call it at an epoch boundary, after the epoch's snapshot was
 * published (the published series keep their last values, as the reference's gauges
 * of a deleted pod do). */
int gpuagg_retire_slots(gpuagg_ctx *ctx, size_t *n_retired);

/* DNS label payload dictionary (utils.AddDNSInfo, flow_utils.go:186-220): interns
 * (rcode, qtypes joined with ",", query, ips joined with ",", num_answers) and
 * returns the id the producer writes into the dns_id column. */
int gpuagg_dns_intern(gpuagg_ctx *ctx, uint32_t rcode, const char *qtypes_joined,
                      const char *query, const char *ips_joined, uint32_t num_answers,
                      uint32_t *dns_id);

/* DNS id lifecycle (the dictionary would otherwise only grow under rotating answers).
 * Over the n contexts of a node (one dictionary interned alike on each, as the Go
 * plugin does; else GPUAGG_EINVAL): aggregates every submitted batch, then finds the DNS
 * ids no DNS group-by key of any of them references -- after an epoch reset
 * (gpuagg_reset, or the non-target side of a merge) that is every id.  Two phases: such
 * an id turns idle; an id still idle at the NEXT call (unreferenced at both, and not
 * handed out again by gpuagg_dns_intern in between) is retired.  Retired ids are reused
 * by later interns, so the caller drops them from its own payload -> id cache: the first
 * min(n_retired, cap) are written to ids.  A record converted with an id before one call
 * and submitted after the next may name a retired id: its group-by entries are then not
 * rendered and count as lost updates (gpuagg_result_dropped).  The reference keeps a DNS
 * series' labels until the metric object is re-created (dns.go:240-242 Clean on
 * reconcile, metrics_module.go:204-214). */
int gpuagg_dns_retire(gpuagg_ctx *const *ctxs, size_t n, uint32_t *ids, size_t cap, size_t *n_retired);

/* ------------------------------------------------------------------------------
 * Records: one decoded flow per row, struct-of-arrays, all uint32.
 *
 *  src_ip, dst_ip  IPv4 as the u32 read little-endian from the 4 network-order
 *                  address bytes (struct packet.src_ip, conntrack.c:37-38; the value
 *                  utils.Int2ip turns into "a.b.c.d", utils_linux.go:51-55)
 *  bytes           RetinaMetadata.Bytes (utils.PacketSize, flow_utils.go:267-274)
 *  meta            bits  0-7  L4 protocol (6 TCP, 17 UDP, other: no L4)
 *                  bits  8-15 verdict passed to utils.ToFlow (1 FORWARDED, 2 DROPPED,
 *                             15 RETRANSMISSION, 16 DNS; flow_utils.go:19-21); 0 means
 *                             FORWARDED, as ToFlow maps it (flow_utils.go:94-96)
 *                  bits 16-17 flow.TrafficDirection (0 UNKNOWN, 1 INGRESS, 2 EGRESS)
 *                  bits 18-20 RetinaMetadata.DropReason (metadata_linux.pb.go:76-84)
 *                  bits 21-26 TCP flags FIN,SYN,RST,PSH,ACK,URG (types_linux.go:22-31)
 *                  bit  27    IsReply
 *                  bits 28-29 RetinaMetadata.DnsType (0 UNKNOWN, 1 QUERY, 2 RESPONSE)
 *                  bits 30-31 observation point passed to ToFlow, values 0-3
 *                             (2 FROM_NETWORK, 3 TO_NETWORK; flow_utils.go:72-92); any
 *                             other point is written as 0 (only 2 and 3 are read)
 *  ports           source port | destination port << 16 (host order, as in flow.L4)
 *  dns_id          gpuagg_dns_intern id (DNS verdict rows only; 0xFFFFFFFF reserved)
 *  tcp_id          RetinaMetadata.TcpId: TSval on TO_NETWORK, TSecr on FROM_NETWORK,
 *                  else 0 (packetparser_linux.go:622-628)
 *  time_ns         the record time ToFlow receives (flow.Time; u64 nanoseconds)
 * ports / dns_id / tcp_id / time_ns may be NULL when no enabled metric reads them
 * (tcp_id and time_ns: the node-apiserver latency metrics).
 * ---------------------------------------------------------------------------- */
typedef struct gpuagg_columns {
  uint32_t *src_ip;
  uint32_t *dst_ip;
  uint32_t *bytes;
  uint32_t *meta;
  uint32_t *ports;
  uint32_t *dns_id;
  uint32_t *tcp_id;
  uint64_t *time_ns;
} gpuagg_columns;

/* Library-owned pinned host batch (the enricher's input ring, enricher.go:45). */
typedef struct gpuagg_batch {
  gpuagg_columns cols;
  size_t capacity;
} gpuagg_batch;

int gpuagg_alloc_batch(gpuagg_ctx *ctx, size_t capacity, gpuagg_batch **out);
void gpuagg_free_batch(gpuagg_ctx *ctx, gpuagg_batch *batch);

/* Host-fed submit: copies n rows to HBM and enqueues the aggregation.  Returns once
 * the batch's host buffers may be refilled (its H2D copies are complete); the
 * aggregation itself runs async.  Two device staging buffers alternate, so the copy of
 * the next batch (on a copy stream) overlaps the aggregation of this one. */
int gpuagg_submit(gpuagg_ctx *ctx, gpuagg_batch *batch, size_t n);

/* Device-resident submit: the columns already live in this ctx's device memory. */
int gpuagg_submit_device(gpuagg_ctx *ctx, const gpuagg_columns *dev_cols, size_t n);

/* ------------------------------------------------------------------------------
 * Raw perf records: the producers' eBPF output structs, decoded on
 * the GPU into the columns above instead of by the Go workers' binary.Read + ToFlow.
 *
 *  GPUAGG_RAW_PACKET  struct packet of packetparser, 72 bytes little-endian
 *                     (pkg/plugin/conntrack/_cprog/conntrack.c:34-49), decoded as
 *                     packetParser.processRecord (packetparser_linux.go:571-631):
 *                     verdict FORWARDED, TrafficDirection = traffic_direction,
 *                     IsReply = is_reply != 0, TCP flags for proto 6 only, ports
 *                     byte-swapped (utils.HostToNetShort, utils_linux.go:65-70).
 *  GPUAGG_RAW_DROP    struct packet of dropreason, 32 bytes little-endian
 *                     (pkg/plugin/dropreason/_cprog/drop_reason.c:39-54), decoded as
 *                     dropReason.processRecord (dropreason_linux.go:345-386): verdict
 *                     DROPPED, INGRESS (obs 2), DropReason = drop_type, Bytes = skb_len.
 *
 * Raw buffers are n back-to-back records (RawSample payloads), 16-byte aligned.
 * A traffic_direction > 3 or drop_type > 7 does not fit the meta word (the eBPF
 * programs emit 0..2 and 0..6): such a row gets verdict 255, which no metric consumes
 * (the sketches still count its 5-tuple), and is counted in
 * gpuagg_stats.decode_out_of_range (read at gpuagg_sync); a host re-renders it.
 * ---------------------------------------------------------------------------- */
#define GPUAGG_RAW_PACKET 1
#define GPUAGG_RAW_DROP 2
#define GPUAGG_RAW_PACKET_SIZE 72
#define GPUAGG_RAW_DROP_SIZE 32

/* Decode only: device raw records -> caller's device columns (ports / dns_id may be
 * NULL; dns_id is filled with 0xFFFFFFFF).  Async on the ctx's stream. */
int gpuagg_decode_device(gpuagg_ctx *ctx, int kind, const void *dev_raw, size_t n,
                         const gpuagg_columns *dev_out);
/* Decode device raw records into the ctx's own columns and aggregate them (async). */
int gpuagg_submit_raw_device(gpuagg_ctx *ctx, int kind, const void *dev_raw, size_t n);
/* Host-fed: copies n raw records (72 or 32 B each) to HBM, decodes and aggregates;
 * returns once host_raw may be reused (the packetparser/dropreason reader's batch). */
int gpuagg_submit_raw(gpuagg_ctx *ctx, int kind, const void *host_raw, size_t n);

/* Multi-GPU sharding on the host (retina_amd/dist.py shard_of): the device
 * of each record, fmix64 of the direction-free 5-tuple (the two (ip, port) ends ordered,
 * so a request and its reply meet on one device for the latency join) mod n_shards.
 * gpuagg_shard_raw reads the fields at their fixed offsets of the raw perf records
 * (GPUAGG_RAW_*: ports byte-swapped as the decode does), gpuagg_shard_columns decoded
 * columns (ports may be NULL: port 0).  Host memory; no ctx or device needed. */
int gpuagg_shard_raw(int kind, const void *raw, size_t n, uint32_t n_shards, uint32_t *shard_out);
int gpuagg_shard_columns(const uint32_t *src_ip, const uint32_t *dst_ip, const uint32_t *ports,
                         const uint32_t *meta, size_t n, uint32_t n_shards, uint32_t *shard_out);

/* Decoded records back to back (the Go plugin's Record, gpuagg_linux.go): the feed kind
 * GPUAGG_RECORD takes arrays of these, shards them by gpuagg_shard_columns' function and
 * transposes them into each context's pinned SoA batch (gpuagg_submit when full). */
#define GPUAGG_RECORD 3
typedef struct gpuagg_record {
  uint32_t src_ip, dst_ip, bytes, meta, ports, dns_id, tcp_id, pad_;
  uint64_t time_ns;
} gpuagg_record;

/* Node-wide raw ingestion (the Go plugin's raw path, gpuagg_linux.go Start/submitRaw):
 * one call shards a buffer of back-to-back raw samples over the node's contexts (one per
 * device; the gpuagg_shard_raw function) into each context's pinned staging of `capacity`
 * records, in input order.  Replaces the packetparser_linux.go:556-654 reader loop's
 * hand-over to its two decode goroutines (:669-696) and the per-record Go re-append.
 *  - Two pinned stagings per context: a full one is submitted without waiting for its
 *    H2D DMA (the call returns once the copy is enqueued) while the other fills; a
 *    staging is refilled only after its own copy-done event.
 *  - The work of a put is split over the feed's host threads (default 4 for one context,
 *    16 for several, at most the cores): shard, then scatter at per-thread prefix
 *    positions through cache-resident tiles.
 *  - Raw kinds are copied as they are and decoded on the GPU (GPUAGG_FEED_RAW_DMA, the
 *    default: one memcpy per sample on the host) or decoded on those threads into pinned
 *    SoA columns (GPUAGG_FEED_HOST_DECODE: only the columns the metric plan reads cross
 *    PCIe, 16 B per record for forward/drop instead of the 72-byte sample; rows counted in
 *    gpuagg_stats.decoded / decode_out_of_range at put).  Both give the same columns.
 * _flush submits every partial staging (the plugin's flushInterval tick and Stop);
 * _submitted reports the records handed to each context.  Not thread-safe: one feed per
 * reader goroutine.  gpuagg_destroy of a context detaches its feeds: their puts and
 * flushes then return GPUAGG_ESTATE, and _destroy still releases them. */
typedef struct gpuagg_raw_feed gpuagg_raw_feed;
#define GPUAGG_FEED_HOST_DECODE 0
#define GPUAGG_FEED_RAW_DMA 1
/* or'ed into a mode (diagnostics): full stagings are counted as submitted but never copied
 * or aggregated -- the host side alone (shard, scatter, host decode into pinned memory),
 * for the node-level host ceiling with the DMA out of the loop */
#define GPUAGG_FEED_DRY_RUN 0x100
/* kind: GPUAGG_RAW_PACKET / GPUAGG_RAW_DROP (perf samples) or GPUAGG_RECORD (gpuagg_record) */
int gpuagg_raw_feed_create(gpuagg_ctx *const *ctxs, size_t n_ctx, int kind, size_t capacity,
                           gpuagg_raw_feed **out);
/* threads: host threads per put (0: keep); mode: GPUAGG_FEED_* (raw kinds; ignored for
 * GPUAGG_RECORD).  Only on an empty feed (after create or _flush), else GPUAGG_ESTATE. */
int gpuagg_raw_feed_configure(gpuagg_raw_feed *feed, uint32_t threads, int mode);
int gpuagg_raw_feed_put(gpuagg_raw_feed *feed, const void *raw, size_t n);
int gpuagg_raw_feed_flush(gpuagg_raw_feed *feed);
int gpuagg_raw_feed_submitted(const gpuagg_raw_feed *feed, uint64_t *per_ctx, size_t n_ctx);
void gpuagg_raw_feed_destroy(gpuagg_raw_feed *feed);

/* Wait for every submitted batch. */
int gpuagg_sync(gpuagg_ctx *ctx);

/* Zeroes every accumulated counter, table entry and sketch register, keeping the
 * metric plan, endpoints and dictionaries (used after a multi-GPU epoch merge). */
int gpuagg_reset(gpuagg_ctx *ctx);

/* Single-process multi-GPU merge (the Go agent drives every GPU of the node from one
 * process): folds the state of ctxs[1..n) into ctxs[0] -- dense counters and count-min
 * summed, HLL registers max-ed, group-by entries inserted-and-added -- over peer copies
 * (xGMI between MI355X devices), then resets ctxs[1..n).  Every ctx must have the same
 * metric plan and the same slot / DNS dictionaries (fed the same cache updates in the
 * same order).  The one-process-per-GPU equivalent is retina_amd/dist.py (RCCL). */
int gpuagg_merge(gpuagg_ctx *const *ctxs, size_t n);

/* ------------------------------------------------------------------------------
 * Output: the Prometheus series the reference's GaugeVec/CounterVec would hold
 * (names under namespace "networkobservability", prometheusexporter.go:11,46-66).
 * Values are exact uint64 (the reference's float64 is exact below 2^53).
 * ---------------------------------------------------------------------------- */
typedef struct gpuagg_result gpuagg_result;

int gpuagg_snapshot(gpuagg_ctx *ctx, gpuagg_result **out);
size_t gpuagg_result_count(const gpuagg_result *r);
int gpuagg_result_series(const gpuagg_result *r, size_t i, const char **metric,
                         uint32_t *n_labels, const char *const **label_names,
                         const char *const **label_values, uint64_t *value);
/* The series' Prometheus family: type "gauge" or "counter" and Help text, as the
 * reference's Init creates the vector (forward.go:18-26,47-64, drops.go:18-23,42-60,
 * tcpflags.go:18-24,43-51, tcpretrans.go:18-24,43-51 -- GaugeVec; dns.go:21-30,50-66 --
 * CounterVec; exporter.CreatePrometheus{Gauge,Counter}VecForMetric,
 * prometheusexporter.go:46-66). */
int gpuagg_result_family(const gpuagg_result *r, size_t i, const char **type, const char **help);
/* Group-by updates lost to a full table since the last reset (0 = every series exact).
 * The snapshot still succeeds; series of the lost updates undercount. */
uint64_t gpuagg_result_dropped(const gpuagg_result *r);
/* Renders the series in the Prometheus text exposition format (0.0.4) exactly as
 * client_golang's registry Gather + expfmt would for the AdvancedRegistry: families
 * sorted by name with # HELP / # TYPE lines, label pairs sorted by name, series sorted by
 * label values, values as Go strconv.FormatFloat(v, 'g', -1, 64).  *len receives the
 * full length; buf (cap bytes, may be NULL) gets the text and a NUL when it fits,
 * else GPUAGG_ECAPACITY. */
int gpuagg_result_render_text(const gpuagg_result *r, char *buf, size_t cap, size_t *len);
/* The same text without a copy: *text points at the result's own NUL-terminated rendering
 * (valid until gpuagg_result_free), *len its length -- for a /metrics handler that writes
 * it out as is (a 13.7M-series exposition is 5 GB: the copy alone is ~0.2 s). */
int gpuagg_result_text(const gpuagg_result *r, const char **text, size_t *len);
void gpuagg_result_free(gpuagg_result *r);

/* ------------------------------------------------------------------------------
 * Sketches (new; no reference code): count-min over the 5-tuple and HyperLogLog
 * of distinct destination IPs per source pod.  Estimates read the state of the
 * last gpuagg_snapshot / gpuagg_sketch_refresh.
 * ---------------------------------------------------------------------------- */
int gpuagg_sketch_refresh(gpuagg_ctx *ctx);
int gpuagg_cms_estimate(gpuagg_ctx *ctx, uint32_t src_ip, uint32_t dst_ip, uint32_t ports,
                        uint32_t proto, uint64_t *estimate);
int gpuagg_hll_estimate(gpuagg_ctx *ctx, int32_t slot, double *estimate);
int gpuagg_cms_copy(gpuagg_ctx *ctx, uint32_t *host_out, size_t n_words);
int gpuagg_hll_copy(gpuagg_ctx *ctx, uint8_t *host_out, size_t n_bytes);

/* ------------------------------------------------------------------------------
 * Multi-GPU merge (one process per GPU).  Mergeable device state is exposed so the
 * caller's collective (RCCL through torch.distributed) can reduce it in place:
 *   dense counters: sum u64      count-min: sum u32      HLL registers: max u8
 * The sparse group-by table is exported as a compact entry list, all-gathered by
 * the caller and imported (insert-or-add) on the merging rank.
 * ---------------------------------------------------------------------------- */
typedef struct gpuagg_state_desc {
  uint64_t *dense_count;   size_t dense_len;    /* u64[dense_len], two arrays */
  uint64_t *dense_bytes;
  uint32_t *cms;           size_t cms_len;      /* u32[cms_len]                */
  uint8_t *hll;            size_t hll_len;      /* u8[hll_len]                 */
  size_t sparse_entry_words;                    /* u64 words per exported entry */
  size_t sparse_len;                            /* group-by table slots (0: none): an
                                                   upper bound on exported entries */
  uint64_t *latency;       size_t latency_len;  /* node-apiserver latency histograms, counts,
                                                   sums, no_response, capacity evictions and
                                                   batches: words [0, 35) sum u64, words
                                                   [35, latency_len) (peak live requests)
                                                   max u64 (NULL / 0 when latency is off)  */
} gpuagg_state_desc;

int gpuagg_state(gpuagg_ctx *ctx, gpuagg_state_desc *out);
/* Compacts the sparse table into dev_out (device u64[cap * sparse_entry_words]);
 * *n_out = entries written.  GPUAGG_ECAPACITY if cap is too small. */
int gpuagg_sparse_export(gpuagg_ctx *ctx, uint64_t *dev_out, size_t cap, size_t *n_out);
/* Inserts-and-adds n exported entries (device pointer) into this ctx's table. */
int gpuagg_sparse_import(gpuagg_ctx *ctx, const uint64_t *dev_in, size_t n);

/* ------------------------------------------------------------------------------
 * Node-apiserver latency (pkg/module/metrics/latency.go).  Enabled by the metric names
 * node_apiserver_latency, node_apiserver_handshake_latency and
 * node_apiserver_no_response in gpuagg_reconcile (utils/metric_names.go:28-30); reads
 * ports, tcp_id, time_ns and the observation point of meta.  The TTL join runs on the
 * GPU per batch (gpuagg_latency.hip); its clock is the running maximum of the record
 * times (the reference's cleaner runs on the wall clock), requests still pending carry
 * over to the next batch.  With latency metrics enabled a submit waits for its batch's
 * event count (one small device-to-host read) before sorting the events.
 * ---------------------------------------------------------------------------- */
/* The apiserver IP set (apiserverWatcherCallbackFn, latency.go:307-346); at most 64. */
int gpuagg_set_apiserver_ips(gpuagg_ctx *ctx, const uint32_t *ipv4, size_t n);

typedef struct gpuagg_latency_state {
  uint32_t enabled;                 /* bit 0 latency, 1 handshake latency, 2 no_response */
  uint64_t latency_buckets[11];     /* per bucket (not cumulative): le 0, 0.5, ..., 4.5, +Inf */
  uint64_t latency_count;
  int64_t latency_sum;              /* ms; observations are integers (math.Round)         */
  uint64_t handshake_buckets[11];
  uint64_t handshake_count;
  int64_t handshake_sum;
  uint64_t no_response;             /* entries that expired unanswered                   */
  uint64_t pending;                 /* requests waiting for a reply (carried over)        */
  uint64_t peak_pending;            /* most requests carried across a batch boundary since
                                       the last reconcile                                  */
  uint64_t peak_live;               /* most requests live at any event since the reset   */
  uint64_t capacity_evictions;      /* requests evicted because `limit` were live when a
                                       new one arrived: ttlcache.WithCapacity(LIMIT)
                                       (latency.go:35,120-121), EvictionReasonCapacityReached,
                                       not a no_response                                 */
  uint64_t capacity_batches;        /* batches in which the capacity bound (replayed in
                                       event order by the sequential pass)              */
  uint64_t limit;                   /* gpuagg_config.latency_limit or 100000             */
} gpuagg_latency_state;

int gpuagg_latency_read(gpuagg_ctx *ctx, gpuagg_latency_state *out);

/* ktime.MonotonicOffset: added to the t_nsec / ts of raw records decoded on the GPU
 * (ToFlow receives MonotonicOffset + T_nsec, packetparser_linux.go:583-585). */
int gpuagg_set_time_offset(gpuagg_ctx *ctx, int64_t ns);

/* ------------------------------------------------------------------------------
 * Enriched-flow emission, standard mode (Enricher.enrich + export, enricher.go:102-140;
 * consumers read them through ExportReader, :189-191): per record, the endpoint that
 * getEndpoint puts into flow.Source / flow.Destination, as the pod's slot (the slot's
 * namespace/name is the cache key of the RetinaEndpoint whose labels and owner
 * references the caller renders), or -1 when the IP is not a pod (service, node or not
 * in the cache: the endpoint stays nil).  Uses the IP -> pod map installed by
 * gpuagg_set_endpoints / gpuagg_cache_commit (GPUAGG_ESTATE before the first one).
 * Async on the ctx's stream, ordered after earlier submits (gpuagg_sync waits).
 * ---------------------------------------------------------------------------- */
int gpuagg_enrich_device(gpuagg_ctx *ctx, const gpuagg_columns *in, size_t n, int32_t *src_slot,
                         int32_t *dst_slot);
/* Host-fed: gpuagg_submit of the batch plus its enriched endpoints, from one H2D copy.
 * The slots (host memory, n each) are written before the call returns; the aggregation
 * may still be running, as after gpuagg_submit.  This is what a plugin with an
 * ExportReader / SetupChannel consumer calls instead of gpuagg_submit. */
int gpuagg_submit_enrich(gpuagg_ctx *ctx, gpuagg_batch *batch, size_t n, int32_t *src_slot,
                         int32_t *dst_slot);

/* ------------------------------------------------------------------------------
 * Hubble-mode L3/L4 enrichment (pkg/hubble/parser/parser_linux.go:64-93,
 * layer34/parser_linux.go:30-84, seven/parser_linux.go:28-146,
 * common/decoder_linux.go:32-60): per record, the source / destination endpoint from the
 * ipcache and the flow summary, as columns; the caller renders flow.Flow objects for
 * Hubble consumers from them (labels and strings stay on the host).
 * ---------------------------------------------------------------------------- */
/* The ipcache image: IP -> identity (ipcache.LookupByIP) and a caller-assigned K8s
 * metadata id (GetK8sMetadata: pod, namespace; 0xFFFFFFFF = none).  Replaces the image. */
int gpuagg_ipcache_set(gpuagg_ctx *ctx, const uint32_t *ipv4, const uint32_t *identity,
                       const uint32_t *meta_id, size_t n);

#define GPUAGG_SUMMARY_NONE 0u  /* no summary                                        */
#define GPUAGG_SUMMARY_TCP 1u   /* "TCP Flags: ..."; arg = flags FIN,SYN,RST,PSH,ACK,URG bits 0-5 */
#define GPUAGG_SUMMARY_UDP 2u   /* "UDP"                                              */
#define GPUAGG_SUMMARY_DROP 3u  /* "Drop Reason: ..."; arg = drop reason              */
#define GPUAGG_SUMMARY_DNS 4u   /* seven.dnsSummary; arg = dns_id | DNS type << 30    */

typedef struct gpuagg_hubble_cols {
  uint32_t *src_identity, *dst_identity;  /* World (2) when the IP is not in the ipcache */
  uint32_t *src_meta, *dst_meta;          /* metadata id, 0xFFFFFFFF = none              */
  uint32_t *summary_kind, *summary_arg;
} gpuagg_hubble_cols;

/* Enriches n records already in device memory (src_ip, dst_ip, meta; dns_id for DNS
 * rows) into the device output columns, async on the ctx's stream (gpuagg_sync waits). */
int gpuagg_hubble_decode_device(gpuagg_ctx *ctx, const gpuagg_columns *in, size_t n,
                                const gpuagg_hubble_cols *out);

/* ------------------------------------------------------------------------------
 * Introspection
 * ---------------------------------------------------------------------------- */
typedef struct gpuagg_stats {
  uint64_t records;          /* rows submitted                                   */
  uint64_t batches;          /* batches submitted                                */
  uint64_t sparse_entries;   /* occupied group-by table entries (at last sync)   */
  uint64_t sparse_dropped;   /* updates lost to a full group-by table (at sync)  */
  uint64_t kernel_launches;  /* timed aggregation launches                       */
  double kernel_ms;          /* summed device time of the aggregation kernel (HIP events) */
  double fold_ms;            /* summed device time of the spill fold kernel          */
  uint32_t last_kernel;      /* kernel of the last launch: GPUAGG_KERNEL_*           */
  uint64_t decoded;          /* raw records decoded on the GPU                       */
  uint64_t decode_out_of_range; /* decoded rows with a field beyond the meta word (at sync) */
  uint64_t decode_launches;  /* timed decode launches                                */
  double decode_ms;          /* summed device time of the decode kernels (HIP events)   */
  uint64_t sketch_launches;  /* timed sketch passes (count-min scatter + fold, HLL)    */
  double sketch_ms;          /* summed device time of the sketch passes              */
  uint64_t async_returns;    /* host-fed submits that returned while their aggregation
                                was still running (the double-buffered overlap)        */
} gpuagg_stats;

#define GPUAGG_KERNEL_NONE 0u          /* nothing launched yet                        */
#define GPUAGG_KERNEL_GENERIC 1u       /* aggregate_kernel: any plan                  */
#define GPUAGG_KERNEL_DENSE_HBM_IP 2u  /* dense_local_kernel: IP table in HBM         */
#define GPUAGG_KERNEL_DENSE_LDS_IP 3u  /* dense_lds_kernel: IP table + u32 bins in LDS */
#define GPUAGG_KERNEL_CPU 4u           /* the CPU backend's host threads               */

/* The timed counters (kernel / fold / sketch / decode ms and launches) are summed from the
 * launches' HIP events when the stats are read (after gpuagg_sync: at once; with launches
 * in flight the call waits for the timed ones), not in gpuagg_sync. */
int gpuagg_get_stats(gpuagg_ctx *ctx, gpuagg_stats *out);
/* Enables HIP-event timing of the aggregation kernel on the ctx's stream; disabling zeroes
 * the timed counters (kernel / fold / sketch / decode ms and launches). */
int gpuagg_set_timing(gpuagg_ctx *ctx, int enabled);
/* Returns the ctx's HIP stream (hipStream_t) as an opaque pointer. */
void *gpuagg_stream(gpuagg_ctx *ctx);
/* Signature of the aggregation kernel of the last launch, spelled as rocprofv3 names it
 * (without "void gpuagg::" and the argument list), e.g. "dense_lds_kernel<2, true, 41u>";
 * "" before the first launch.  Lets a profile be matched to the kernel that ran. */
const char *gpuagg_kernel_name(const gpuagg_ctx *ctx);
/* The same for the last sketch pass: its kernels joined by "+", e.g.
 * "sketch_stage_kernel<true>+cms_fold_kernel+hll_split_kernel+hll_fold_kernel". */
const char *gpuagg_sketch_kernel_name(const gpuagg_ctx *ctx);
/* Hash of the sources this library was built from (retina_amd/build.py): profiles under
 * profiles/ carry it, and bench.py uses a profile's counters only for the same build. */
const char *gpuagg_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* GPUAGG_H */
