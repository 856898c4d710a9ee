// Copyright (c) the retina_amd authors.
//
// Package gpuagg is the Retina plugin that drives the MI355X flow-aggregation engine
// through its C ABI (include/gpuagg.h). It keeps the registry.Plugin interface
// (pkg/plugin/registry/registry.go:16-34) so PluginManager can run it like any other
// plugin, and it replaces the enricher + advanced-metrics goroutines
// (pkg/enricher/enricher.go:68-135, pkg/module/metrics/metrics_module.go:276-305).
//
// One engine context per gfx950 device of the node; records are sharded over them by
// the 5-tuple hash of retina_amd/dist.py (shard_of) and the contexts are merged into the
// first one once per scrape epoch (gpuagg_merge: peer copies over xGMI).
//
// NOTE: the image this repository is built in has no Go toolchain; this file is the
// maintainer-side binding, compiled only inside a Retina tree (build tag gpuagg).
//
//go:build linux && gpuagg

package gpuagg

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../retina_amd -lgpuagg -Wl,-rpath,${SRCDIR}/../../../retina_amd
#include <stdlib.h>
#include "gpuagg.h"
*/
import "C"

import (
	"context"
	"encoding/binary"
	"errors"
	"fmt"
	"io"
	"math/bits"
	"net"
	"os"
	"strconv"
	"strings"
	"sync"
	"time"
	"unsafe"

	"github.com/cilium/cilium/api/v1/flow"
	v1 "github.com/cilium/cilium/pkg/hubble/api/v1"
	api "github.com/microsoft/retina/crd/api/v1alpha1"
	"github.com/microsoft/retina/crd/api/v1alpha1/validations"
	"github.com/microsoft/retina/pkg/common"
	kcfg "github.com/microsoft/retina/pkg/config"
	"github.com/microsoft/retina/pkg/controllers/cache"
	"github.com/microsoft/retina/pkg/exporter"
	"github.com/microsoft/retina/pkg/ktime"
	"github.com/microsoft/retina/pkg/pubsub"
	"github.com/microsoft/retina/pkg/log"
	"github.com/microsoft/retina/pkg/metrics"
	"github.com/microsoft/retina/pkg/plugin/registry"
	"github.com/microsoft/retina/pkg/utils"
	"github.com/prometheus/client_golang/prometheus"
	"go.uber.org/zap"
	"google.golang.org/protobuf/types/known/wrapperspb"
)

const (
	name          = "gpuagg"
	// Pinned host memory per device (INTEGRATION.md "Memory and threads"): each feed keeps
	// two stagings per device.  The packetparser feed carries the traffic: its stagings of
	// 2^22 samples spread a launch's fixed cost (LDS image fill, staged bins) over 4M
	// records; drops, decoded records and the enriched-flow batch are far rarer and get
	// 2^20.  Per device: 2 x 2^22 x 72 B + 2 x 2^20 x 32 B + 2 x 2^20 x 36 B + 2^20 x 36 B
	// = 0.78 GB (RETINA_GPUAGG_PACKET_STAGING_LOG2 = 20 brings it to 0.29 GB).
	packetCapacity = 1 << 22 // raw packetparser samples per staging (default)
	batchCapacity  = 1 << 20 // drop samples / decoded records per staging; enriched-flow batch
	rawPiece      = 1 << 16 // samples / records buffered in Go before each hand-over to Start
	flushInterval = 100 * time.Millisecond
	scrapeEpoch   = 5 * time.Second
	maxSlots      = 1 << 20 // hard cap; dense counters grow with the pods actually seen
	sparseLog2    = 22
	channelDepth  = 10000 // like packetparser's recordsChannel (types_linux.go:37-38)
	pieceDepth    = 16    // full pieces of rawPiece waiting for Start (1M samples)
)

// Record is one decoded flow in the column layout of include/gpuagg.h. Producers
// (packetparser.processRecord, dropReason.processRecord, dns.eventHandler,
// tcpretrans.eventHandler) fill it instead of building a *flow.Flow.
type Record struct {
	SrcIP, DstIP, Bytes, Meta, Ports, DNSID uint32
	TcpID  uint32 // RetinaMetadata.TcpId (latency metrics)
	TimeNs uint64 // the time ToFlow receives (latency metrics)
}

// Raw perf-record kinds (GPUAGG_RAW_* of include/gpuagg.h): packetparser and
// dropreason hand their perf.Record.RawSample bytes to WriteRaw and skip
// binary.Read + utils.ToFlow (packetparser_linux.go:571-631, dropreason_linux.go:345-386);
// the engine decodes them on the GPU.
const (
	RawPacket = int(C.GPUAGG_RAW_PACKET) // 72-byte struct packet, conntrack.c:34-49
	RawDrop   = int(C.GPUAGG_RAW_DROP)   // 32-byte struct packet, drop_reason.c:39-54
)

var rawSize = map[int]int{RawPacket: int(C.GPUAGG_RAW_PACKET_SIZE), RawDrop: int(C.GPUAGG_RAW_DROP_SIZE)}

// rawPiece is up to rawPiece back-to-back samples of one kind, handed to Start at once.
type rawSample struct {
	kind int
	b    []byte
}

// rawBatcher collects one kind's samples from the producers (WriteRaw): an append under a
// mutex per sample, one channel operation per rawPiece samples (the reference pays a
// channel operation per sample, packetparser_linux.go:643-651).
type rawBatcher struct {
	mu  sync.Mutex
	buf []byte
}

// device is one engine context and its pinned batch.
type device struct {
	ctx   *C.gpuagg_ctx
	batch *C.gpuagg_batch
	n     int
	cols  [7][]uint32 // src, dst, bytes, meta, ports, dns_id, tcp_id
	times []uint64
}

// packetStaging is the packetparser feed's staging size in samples: packetCapacity, or
// 2^RETINA_GPUAGG_PACKET_STAGING_LOG2 (16..22) for agents under a tight memory limit.
func packetStaging() int {
	if v, err := strconv.Atoi(os.Getenv("RETINA_GPUAGG_PACKET_STAGING_LOG2")); err == nil && v >= 16 && v <= 22 {
		return 1 << v
	}
	return packetCapacity
}

type gpuAgg struct {
	cfg *kcfg.Config
	l   *log.ZapLogger

	// mu serialises every ABI call (one thread per ctx at a time, include/gpuagg.h) and
	// guards the fields below.
	mu       sync.Mutex
	devs     []*device
	feeds    map[int]*C.gpuagg_raw_feed    // per kind: shard + scatter into pinned per-device staging
	recFeed  *C.gpuagg_raw_feed            // decoded records: shard + transpose into pinned SoA batches
	spec     *api.MetricsSpec
	vecs     map[string]*prometheus.GaugeVec
	ctrs     map[string]*prometheus.CounterVec
	ctrLast  map[string]float64 // counter series: value already added
	dirty    bool               // cache changed since the last commit
	version  uint64
	stopping bool

	// enriched-flow emission (SetupChannel): the consumer channel, the cache's endpoint
	// per slot (what getEndpoint copies, enricher.go:142-183), the DNS payload per dns_id
	// (AddDNSInfo's arguments) and the per-batch endpoint slots from gpuagg_submit_enrich
	external   chan *v1.Event
	slotEP     map[int32]*common.RetinaEndpoint
	dnsByID    map[uint32]dnsPayload
	dnsRetired []func([]uint32) // producer caches told about retired ids (Enricher.dropDNS)
	enrichSrc  []int32
	enrichDst  []int32

	// producer side: single Write()s collect in recIn (recMu also orders them against
	// WriteBatch slices), raw samples in a batcher per kind; full pieces go to Start
	recMu   sync.Mutex
	recIn   []Record
	batches chan []Record // record pieces and WriteBatch slices, in arrival order
	rawIn   map[int]*rawBatcher
	raw     chan rawSample // full raw pieces
	rawFree chan []byte    // recycled piece buffers
	done    chan struct{}  // closed when Start returns

	// node-apiserver latency (latency.go): apiserver IP set from the pubsub topic, the
	// histograms as a collector, no_response as a counter vec
	apiIPs     map[string]uint32
	apiSubID   string
	latency    *latencyCollector
	noResponse *prometheus.CounterVec
	noRespLast float64
}

type dnsPayload struct {
	rcode      uint32
	qtypes     []string
	query      string
	ips        []string
	numAnswers uint32
}

// latencyCollector exposes the engine's latency histograms with the reference's names,
// Help texts and buckets (latency.go:28-39, LinearBuckets(0, 0.5, 10)) as const
// histograms built from gpuagg_latency_read.
type latencyCollector struct {
	mu      sync.Mutex
	st      C.gpuagg_latency_state
	lat, hs *prometheus.Desc
}

func newLatencyCollector() *latencyCollector {
	ns := exporter.RetinaNamespace
	return &latencyCollector{
		lat: prometheus.NewDesc(ns+"_adv_node_apiserver_latency", "Latency of node apiserver in ms", nil, nil),
		hs: prometheus.NewDesc(ns+"_adv_node_apiserver_tcp_handshake_latency",
			"Latency of node apiserver tcp handshake in ms", nil, nil),
	}
}

func (lc *latencyCollector) Describe(ch chan<- *prometheus.Desc) { ch <- lc.lat; ch <- lc.hs }

func (lc *latencyCollector) Collect(ch chan<- prometheus.Metric) {
	lc.mu.Lock()
	st := lc.st
	lc.mu.Unlock()
	emit := func(d *prometheus.Desc, bk [11]C.uint64_t, cnt C.uint64_t, sum C.int64_t) {
		buckets := map[float64]uint64{}
		acc := uint64(0)
		for i := 0; i < 10; i++ { // cumulative upper bounds 0, 0.5, ..., 4.5 (+Inf = count)
			acc += uint64(bk[i])
			buckets[0.5*float64(i)] = acc
		}
		ch <- prometheus.MustNewConstHistogram(d, uint64(cnt), float64(sum), buckets)
	}
	if st.enabled&1 != 0 {
		emit(lc.lat, st.latency_buckets, st.latency_count, st.latency_sum)
	}
	if st.enabled&2 != 0 {
		emit(lc.hs, st.handshake_buckets, st.handshake_count, st.handshake_sum)
	}
}

var (
	instance   *gpuAgg
	instanceMu sync.Mutex
)

func init() {
	registry.Add(name, New)
}

// New is the registry.PluginFunc (registry.go:37).
func New(cfg *kcfg.Config) registry.Plugin {
	g := &gpuAgg{cfg: cfg, l: log.Logger().Named(name),
		raw: make(chan rawSample, pieceDepth), rawFree: make(chan []byte, pieceDepth),
		rawIn:   map[int]*rawBatcher{RawPacket: {}, RawDrop: {}},
		batches: make(chan []Record, channelDepth/64+1)}
	instanceMu.Lock()
	instance = g
	instanceMu.Unlock()
	return g
}

// Instance returns the plugin for producers and the cache tee (nil before New).
func Instance() *gpuAgg {
	instanceMu.Lock()
	defer instanceMu.Unlock()
	return instance
}

func (g *gpuAgg) Name() string                       { return name }
func (g *gpuAgg) Generate(ctx context.Context) error { return nil }
func (g *gpuAgg) Compile(ctx context.Context) error  { return nil }

// SetupChannel registers a consumer of the enriched flows (packetparser's external
// channel, packetparser_linux.go:335-338,642-651; the enricher's export to ExportReader,
// enricher.go:137-140,189-191).  From then on every batch is submitted with
// gpuagg_submit_enrich, whose per-record endpoint slots become flow.Source /
// flow.Destination; sends never block, a full channel counts a lost event.
func (g *gpuAgg) SetupChannel(c chan *v1.Event) error {
	g.mu.Lock()
	defer g.mu.Unlock()
	g.external = c
	if c != nil && g.enrichSrc == nil {
		g.enrichSrc = make([]int32, batchCapacity)
		g.enrichDst = make([]int32, batchCapacity)
	}
	return nil
}

// endpointLocked is getEndpoint for a slot (-1: the IP is not a pod, the endpoint stays nil).
func (g *gpuAgg) endpointLocked(slot int32) *flow.Endpoint {
	ep := g.slotEP[slot]
	if slot < 0 || ep == nil {
		return nil
	}
	var wl []*flow.Workload
	if refs := ep.OwnerRefs(); refs != nil {
		wl = make([]*flow.Workload, 0, len(refs))
		for _, r := range refs {
			wl = append(wl, &flow.Workload{Name: r.Name, Kind: r.Kind})
		}
	}
	return &flow.Endpoint{Namespace: ep.Namespace(), PodName: ep.Name(), Labels: ep.FormattedLabels(), Workloads: wl}
}

// emitLocked rebuilds the producer's flow.Flow of each of the device's n records (the
// fields packetparser / dropreason / dns / tcpretrans set, packetparser_linux.go:583-628)
// with the enriched endpoints and sends it to the external channel.
func (g *gpuAgg) emitLocked(d *device, n int) {
	for i := 0; i < n; i++ {
		m := d.cols[3][i]
		ports := d.cols[4][i]
		verdict := flow.Verdict((m >> 8) & 0xff)
		fl := utils.ToFlow(g.l, int64(d.times[i]), utils.Int2ip(d.cols[0][i]).To4(), utils.Int2ip(d.cols[1][i]).To4(),
			ports&0xffff, ports>>16, uint8(m&0xff), uint8(m>>30), verdict)
		if fl == nil {
			continue
		}
		fl.IsReply = &wrapperspb.BoolValue{Value: (m>>27)&1 == 1}
		fl.TrafficDirection = flow.TrafficDirection((m >> 16) & 3)
		meta := &utils.RetinaMetadata{}
		utils.AddPacketSize(meta, d.cols[2][i])
		f := uint16((m >> 21) & 0x3f) // FIN, SYN, RST, PSH, ACK, URG
		utils.AddTCPFlags(fl, (f>>1)&1, (f>>4)&1, f&1, (f>>2)&1, (f>>3)&1, (f>>5)&1)
		if verdict == flow.Verdict_DROPPED {
			utils.AddDropReason(fl, meta, uint16((m>>18)&7))
		}
		if id := d.cols[6][i]; id != 0 {
			utils.AddTCPID(meta, uint64(id))
		}
		if t := (m >> 28) & 3; t != 0 {
			if p, ok := g.dnsByID[d.cols[5][i]]; ok {
				qr := "Q"
				if t == 2 {
					qr = "R"
				}
				utils.AddDNSInfo(fl, meta, qr, p.rcode, p.query, p.qtypes, int(p.numAnswers), p.ips)
			}
		}
		utils.AddRetinaMetadata(fl, meta)
		fl.Source = g.endpointLocked(g.enrichSrc[i])
		fl.Destination = g.endpointLocked(g.enrichDst[i])
		select {
		case g.external <- &v1.Event{Event: fl, Timestamp: fl.GetTime()}:
		default:
			metrics.LostEventsCounter.WithLabelValues(utils.ExternalChannel, name).Inc()
		}
	}
}

func lastError(ctx *C.gpuagg_ctx) string { return C.GoString(C.gpuagg_last_error(ctx)) }

func check(ctx *C.gpuagg_ctx, rc C.int, what string) error {
	if rc != C.GPUAGG_OK {
		return fmt.Errorf("%s: %d: %s", what, int(rc), lastError(ctx))
	}
	return nil
}

// each applies fn to every device context; the first error wins.
func (g *gpuAgg) each(what string, fn func(ctx *C.gpuagg_ctx) C.int) error {
	var err error
	for _, d := range g.devs {
		if e := check(d.ctx, fn(d.ctx), what); e != nil && err == nil {
			err = e
		}
	}
	return err
}

// Init creates one engine context per gfx950 device (PluginManager calls Stop before
// Init on every reconcile, pluginmanager.go:91-112).  A node without one gets a single
// context on the library's CPU backend (GPUAGG_FLAG_CPU_BACKEND: the same plan and
// results on host threads), so advanced metrics exist on every node as the reference's
// CPU loop provides them (metrics_module.go:276-317).
func (g *gpuAgg) Init() error {
	g.mu.Lock()
	defer g.mu.Unlock()
	var ndev C.int
	flags := C.uint32_t(0)
	if rc := C.gpuagg_device_count(&ndev); rc != C.GPUAGG_OK || ndev == 0 {
		g.l.Warn("gpuagg: no MI355X (gfx950) device: aggregating on the CPU backend")
		ndev, flags = 1, C.GPUAGG_FLAG_CPU_BACKEND
	}
	remote := C.int32_t(0)
	if g.cfg.RemoteContext {
		remote = 1
	}
	for dev := 0; dev < int(ndev); dev++ {
		cfg := C.gpuagg_config{
			abi_version: C.GPUAGG_ABI_VERSION, device: C.int32_t(dev), remote_context: remote,
			max_slots: maxSlots, max_ips: 2 * maxSlots, sparse_capacity_log2: sparseLog2, flags: flags,
		}
		d := &device{}
		if rc := C.gpuagg_create(&cfg, &d.ctx); rc != C.GPUAGG_OK {
			g.destroyLocked()
			return fmt.Errorf("gpuagg_create(device %d): %d", dev, int(rc))
		}
		if err := check(d.ctx, C.gpuagg_alloc_batch(d.ctx, batchCapacity, &d.batch), "gpuagg_alloc_batch"); err != nil {
			C.gpuagg_destroy(d.ctx)
			g.destroyLocked()
			return err
		}
		c := d.batch.cols
		col := func(p *C.uint32_t) []uint32 { return unsafe.Slice((*uint32)(unsafe.Pointer(p)), batchCapacity) }
		d.cols = [7][]uint32{col(c.src_ip), col(c.dst_ip), col(c.bytes), col(c.meta), col(c.ports), col(c.dns_id),
			col(c.tcp_id)}
		d.times = unsafe.Slice((*uint64)(unsafe.Pointer(c.time_ns)), batchCapacity)
		// raw records carry boot-time stamps; ToFlow adds ktime.MonotonicOffset (packetparser_linux.go:583-585)
		C.gpuagg_set_time_offset(d.ctx, C.int64_t(ktime.MonotonicOffset.Nanoseconds()))
		g.devs = append(g.devs, d)
	}
	// raw perf samples: one library-side feed per kind shards each handed-over buffer over
	// the devices and copies it into their pinned staging (no per-record Go append, no
	// pageable H2D copy)
	ctxs := make([]*C.gpuagg_ctx, len(g.devs))
	for i, d := range g.devs {
		ctxs[i] = d.ctx
	}
	g.feeds = map[int]*C.gpuagg_raw_feed{}
	for kind := range rawSize {
		var f *C.gpuagg_raw_feed
		capacity := C.size_t(batchCapacity)
		if kind == RawPacket {
			capacity = C.size_t(packetStaging())
		}
		if err := check(ctxs[0], C.gpuagg_raw_feed_create(&ctxs[0], C.size_t(len(ctxs)), C.int(kind),
			capacity, &f), "gpuagg_raw_feed_create"); err != nil {
			g.destroyLocked()
			return err
		}
		g.feeds[kind] = f
	}
	// decoded records (Write / WriteBatch) go through a GPUAGG_RECORD feed: one cgo call per
	// slice shards them and transposes them into each device's pinned SoA batch in C (the
	// Record layout is struct gpuagg_record's)
	if unsafe.Sizeof(Record{}) != uintptr(C.sizeof_gpuagg_record) {
		g.destroyLocked()
		return fmt.Errorf("gpuagg: Record is %d bytes, gpuagg_record %d", unsafe.Sizeof(Record{}), int(C.sizeof_gpuagg_record))
	}
	if err := check(ctxs[0], C.gpuagg_raw_feed_create(&ctxs[0], C.size_t(len(ctxs)), C.GPUAGG_RECORD,
		batchCapacity, &g.recFeed), "gpuagg_raw_feed_create(records)"); err != nil {
		g.destroyLocked()
		return err
	}
	g.stopping = false
	g.spec = nil
	g.apiIPs = map[string]uint32{}
	if g.apiSubID == "" {
		fn := pubsub.CallBackFunc(g.apiserverCallback)
		g.apiSubID = pubsub.New().Subscribe(common.PubSubAPIServer, &fn)
	}
	return nil
}

// Reconcile mirrors Module.Reconcile (metrics_module.go:142-203): nothing happens when
// the spec is unchanged or only its namespaces changed (validations.MetricsContextOptionsCompare);
// otherwise the AdvancedRegistry is reset and the engine re-plans its metric groups.
func (g *gpuAgg) Reconcile(spec *api.MetricsSpec) error {
	g.mu.Lock()
	defer g.mu.Unlock()
	if g.spec != nil && (g.spec.Equals(spec) ||
		validations.MetricsContextOptionsCompare(g.spec.ContextOptions, spec.ContextOptions)) {
		g.spec = spec
		return nil
	}
	opts := make([]C.gpuagg_metric_options, len(spec.ContextOptions))
	var frees []unsafe.Pointer
	defer func() {
		for _, p := range frees {
			C.free(p)
		}
	}()
	cstrs := func(ss []string) (**C.char, C.uint32_t, C.int32_t) {
		if ss == nil {
			return nil, 0, 0
		}
		arr := C.malloc(C.size_t(len(ss)+1) * C.size_t(unsafe.Sizeof(uintptr(0))))
		frees = append(frees, arr)
		view := unsafe.Slice((**C.char)(arr), len(ss)+1)
		for i, s := range ss {
			cs := C.CString(s)
			frees = append(frees, unsafe.Pointer(cs))
			view[i] = cs
		}
		return (**C.char)(arr), C.uint32_t(len(ss)), 1
	}
	for i, o := range spec.ContextOptions {
		n := C.CString(o.MetricName)
		frees = append(frees, unsafe.Pointer(n))
		opts[i].metric_name = n
		opts[i].source_labels, opts[i].n_source_labels, opts[i].source_labels_set = cstrs(o.SourceLabels)
		opts[i].destination_labels, opts[i].n_destination_labels, opts[i].destination_labels_set = cstrs(o.DestinationLabels)
	}
	var p *C.gpuagg_metric_options
	if len(opts) > 0 {
		p = &opts[0]
	}
	if err := g.each("gpuagg_reconcile", func(ctx *C.gpuagg_ctx) C.int {
		return C.gpuagg_reconcile(ctx, p, C.size_t(len(opts)))
	}); err != nil {
		return err
	}
	exporter.ResetAdvancedMetricsRegistry()
	g.vecs = map[string]*prometheus.GaugeVec{}
	g.ctrs = map[string]*prometheus.CounterVec{}
	g.ctrLast = map[string]float64{}
	g.latency, g.noResponse, g.noRespLast = nil, nil, 0
	for _, o := range spec.ContextOptions {
		switch o.MetricName { // NewLatencyMetrics (latency.go:73-115)
		case utils.NodeAPIServerLatencyName, utils.NodeAPIServerTCPHandshakeLatencyName:
			if g.latency == nil {
				g.latency = newLatencyCollector()
				exporter.AdvancedRegistry.MustRegister(g.latency)
			}
		case utils.NoResponseFromAPIServerName:
			g.noResponse = exporter.CreatePrometheusCounterVecForMetric(exporter.AdvancedRegistry,
				"adv_node_apiserver_no_response", "Number of packets that did not get a response from node apiserver",
				"no_response")
		}
	}
	g.spec = spec
	return nil
}

// apiserverCallback mirrors apiserverWatcherCallbackFn (latency.go:307-346): the
// apiserver IP set follows the cache's add / delete events and is handed to every device.
func (g *gpuAgg) apiserverCallback(obj interface{}) {
	event, ok := obj.(*cache.CacheEvent)
	if !ok || event == nil {
		return
	}
	apiServer, ok := event.Obj.(*common.APIServerObject)
	if !ok || apiServer == nil {
		return
	}
	g.mu.Lock()
	defer g.mu.Unlock()
	for _, ip := range apiServer.IPs() {
		v4 := ip.To4()
		if v4 == nil {
			continue
		}
		switch event.Type {
		case cache.EventTypeAddAPIServerIPs:
			g.apiIPs[v4.String()] = binary.LittleEndian.Uint32(v4) // the LE u32 of the record columns
		case cache.EventTypeDeleteAPIServerIPs:
			delete(g.apiIPs, v4.String())
		}
	}
	ips := make([]C.uint32_t, 0, len(g.apiIPs))
	for _, v := range g.apiIPs {
		ips = append(ips, C.uint32_t(v))
	}
	var p *C.uint32_t
	if len(ips) > 0 {
		p = &ips[0]
	}
	if err := g.each("gpuagg_set_apiserver_ips", func(ctx *C.gpuagg_ctx) C.int {
		return C.gpuagg_set_apiserver_ips(ctx, p, C.size_t(len(ips)))
	}); err != nil {
		g.l.Error("apiserver ips", zap.Error(err))
	}
}

// Write is what producers call per decoded record (Enricher.Write's replacement). It
// never blocks the reader: records collect in recIn and go to Start rawPiece at a time; a
// full channel drops the piece and counts it, like packetparser's readData
// (packetparser_linux.go:643-651,689-695).
func (g *gpuAgg) Write(r Record) {
	g.recMu.Lock()
	g.recIn = append(g.recIn, r)
	if len(g.recIn) >= rawPiece {
		g.sendRecordsLocked(g.recIn)
		g.recIn = nil
	}
	g.recMu.Unlock()
}

// WriteBatch hands over a slice of decoded records with one channel operation (a
// producer draining several perf records per wake-up); the slice is owned by the plugin
// afterwards.  Records of earlier Write()s go first (the latency join pairs a request
// with the reply after it).  A full channel drops the whole slice and counts every record.
func (g *gpuAgg) WriteBatch(rs []Record) {
	if len(rs) == 0 {
		return
	}
	g.recMu.Lock()
	defer g.recMu.Unlock()
	if len(g.recIn) > 0 {
		g.sendRecordsLocked(g.recIn)
		g.recIn = nil
	}
	g.sendRecordsLocked(rs)
}

func (g *gpuAgg) sendRecordsLocked(rs []Record) {
	select {
	case g.batches <- rs:
	default:
		metrics.LostEventsCounter.WithLabelValues(utils.BufferedChannel, name).Add(float64(len(rs)))
	}
}

// WriteRaw takes one perf RawSample of the given kind; a sample of the wrong size is
// refused like binary.Read's size mismatch (dropreason_linux.go:347-352).  Samples are
// appended to the kind's piece (one copy, under a mutex); every rawPiece samples the piece
// goes to Start with one channel operation.
func (g *gpuAgg) WriteRaw(kind int, sample []byte) error {
	sz, ok := rawSize[kind]
	if !ok || len(sample) != sz {
		return fmt.Errorf("gpuagg: raw sample of %d bytes for kind %d", len(sample), kind)
	}
	b := g.rawIn[kind]
	b.mu.Lock()
	if b.buf == nil {
		b.buf = g.rawBuffer()
	}
	b.buf = append(b.buf, sample...)
	if len(b.buf) >= rawPiece*sz {
		g.sendRaw(kind, b.buf)
		b.buf = nil
	}
	b.mu.Unlock()
	return nil
}

// sendRaw hands a piece to Start (non-blocking: a full channel drops it and counts its samples).
func (g *gpuAgg) sendRaw(kind int, buf []byte) {
	select {
	case g.raw <- rawSample{kind, buf}:
	default:
		metrics.LostEventsCounter.WithLabelValues(utils.BufferedChannel, name).Add(float64(len(buf) / rawSize[kind]))
		g.recycleRaw(buf)
	}
}

func (g *gpuAgg) rawBuffer() []byte {
	select {
	case b := <-g.rawFree:
		return b[:0]
	default:
		return make([]byte, 0, rawPiece*int(C.GPUAGG_RAW_PACKET_SIZE))
	}
}

func (g *gpuAgg) recycleRaw(b []byte) {
	select {
	case g.rawFree <- b:
	default: // enough spares
	}
}

// flushProducers moves the partial pieces (records, each raw kind) to Start's channels,
// behind everything already queued, so the flush that follows keeps arrival order.
func (g *gpuAgg) flushProducers() {
	g.recMu.Lock()
	if len(g.recIn) > 0 {
		g.sendRecordsLocked(g.recIn)
		g.recIn = nil
	}
	g.recMu.Unlock()
	for kind, b := range g.rawIn {
		b.mu.Lock()
		if len(b.buf) > 0 {
			g.sendRaw(kind, b.buf)
			b.buf = nil
		}
		b.mu.Unlock()
	}
}

// shardOf is retina_amd/dist.py shard_of and the library's gpuagg_shard_columns (whose
// agreement is tests/test_cpu_shard.py): fmix64 of the direction-free 5-tuple (the
// (ip, port) ends in order, so a request and its reply meet on one device for the
// latency join), mod the devices.  Restated in Go so the per-record path needs no cgo call.
func shardOf(r *Record, n int) int {
	if n == 1 {
		return 0
	}
	fmix := func(k uint64) uint64 {
		k ^= k >> 33
		k *= 0xff51afd7ed558ccd
		k ^= k >> 33
		k *= 0xc4ceb9fe1a85ec53
		k ^= k >> 33
		return k
	}
	a, b := uint64(r.SrcIP)<<16|uint64(r.Ports&0xffff), uint64(r.DstIP)<<16|uint64(r.Ports>>16)
	if a > b {
		a, b = b, a
	}
	return int(fmix(a^fmix(b^(uint64(r.Meta&0xff)<<48)^0x1F2E3D4C5B6A7988)) % uint64(n))
}

// Start blocks until ctx is done (PluginManager runs it in an errgroup goroutine,
// pluginmanager.go:166-169).  It owns the pinned batches; Stop waits for it to return
// before the contexts are destroyed.
func (g *gpuAgg) Start(ctx context.Context) error {
	g.mu.Lock()
	if len(g.devs) == 0 || g.stopping {
		g.mu.Unlock()
		return errors.New("gpuagg: Start before Init")
	}
	g.done = make(chan struct{})
	devs := g.devs
	g.mu.Unlock()
	defer close(g.done)

	flush := time.NewTicker(flushInterval)
	epoch := time.NewTicker(scrapeEpoch)
	defer flush.Stop()
	defer epoch.Stop()
	submit := func(d *device) error {
		if d.n == 0 {
			return nil
		}
		g.mu.Lock()
		defer g.mu.Unlock()
		if err := g.commitLocked(); err != nil {
			return err
		}
		if g.external != nil {
			// one H2D copy for both: the aggregation and the records' endpoint slots
			err := check(d.ctx, C.gpuagg_submit_enrich(d.ctx, d.batch, C.size_t(d.n),
				(*C.int32_t)(unsafe.Pointer(&g.enrichSrc[0])), (*C.int32_t)(unsafe.Pointer(&g.enrichDst[0]))),
				"gpuagg_submit_enrich")
			if err == nil {
				g.emitLocked(d, d.n)
			}
			d.n = 0
			return err
		}
		// returns once the H2D copy is done: the batch may be refilled while the GPU
		// aggregates (double-buffered staging, include/gpuagg.h)
		err := check(d.ctx, C.gpuagg_submit(d.ctx, d.batch, C.size_t(d.n)), "gpuagg_submit")
		d.n = 0
		return err
	}
	// putRaw hands one piece of a kind's samples to its feed: the library shards them by
	// the 5-tuple at the records' fixed offsets (conntrack.c:34-49, drop_reason.c:39-54;
	// the function of shardOf and dist.shard_of, so a flow's raw and decoded records meet
	// on one device) and copies each into its device's pinned staging, starting the DMA of
	// the stagings that fill; the piece's buffer is recycled once the call returns.
	putRaw := func(s rawSample) error {
		defer g.recycleRaw(s.b)
		g.mu.Lock()
		defer g.mu.Unlock()
		if err := g.commitLocked(); err != nil {
			return err
		}
		if len(s.b) == 0 {
			return nil
		}
		return check(devs[0].ctx, C.gpuagg_raw_feed_put(g.feeds[s.kind], unsafe.Pointer(&s.b[0]),
			C.size_t(len(s.b)/rawSize[s.kind])), "gpuagg_raw_feed_put")
	}
	// putRecords hands a slice of decoded records to the record feed (the enriched-flow
	// path keeps the per-record batches: emitLocked rebuilds flows from them)
	putRecords := func(rs []Record) error {
		g.mu.Lock()
		defer g.mu.Unlock()
		if err := g.commitLocked(); err != nil {
			return err
		}
		if len(rs) == 0 {
			return nil
		}
		return check(devs[0].ctx, C.gpuagg_raw_feed_put(g.recFeed, unsafe.Pointer(&rs[0]), C.size_t(len(rs))),
			"gpuagg_raw_feed_put(records)")
	}
	// put copies one decoded record into its device's pinned batch (device by shardOf)
	put := func(r *Record) {
		d := devs[shardOf(r, len(devs))]
		i := d.n
		d.cols[0][i], d.cols[1][i], d.cols[2][i], d.cols[3][i], d.cols[4][i], d.cols[5][i], d.cols[6][i] =
			r.SrcIP, r.DstIP, r.Bytes, r.Meta, r.Ports, r.DNSID, r.TcpID
		d.times[i] = r.TimeNs
		d.n++
		if d.n == batchCapacity {
			if err := submit(d); err != nil {
				g.l.Error("submit failed", zap.Error(err))
			}
		}
	}
	takeBatch := func(rs []Record) {
		if g.external != nil {
			for i := range rs {
				put(&rs[i])
			}
			return
		}
		if err := putRecords(rs); err != nil {
			g.l.Error("record submit failed", zap.Error(err))
		}
	}
	takeRaw := func(s rawSample) {
		if err := putRaw(s); err != nil {
			g.l.Error("raw submit failed", zap.Error(err))
		}
	}
	// submitAll: the producers' partial pieces join the queues, everything queued is
	// handed over in arrival order, then every partial staging is submitted (flushInterval,
	// the scrape epoch, Stop)
	submitAll := func() error {
		g.flushProducers()
	drain:
		for {
			select {
			case rs := <-g.batches:
				takeBatch(rs)
			case s := <-g.raw:
				takeRaw(s)
			default:
				break drain
			}
		}
		var err error
		for _, d := range devs {
			if e := submit(d); e != nil && err == nil {
				err = e
			}
		}
		g.mu.Lock()
		defer g.mu.Unlock()
		if e := check(devs[0].ctx, C.gpuagg_raw_feed_flush(g.recFeed), "gpuagg_raw_feed_flush(records)"); e != nil && err == nil {
			err = e
		}
		for kind := range rawSize {
			if e := check(devs[0].ctx, C.gpuagg_raw_feed_flush(g.feeds[kind]), "gpuagg_raw_feed_flush"); e != nil && err == nil {
				err = e
			}
		}
		return err
	}
	for {
		select {
		case <-ctx.Done():
			return submitAll()
		case rs := <-g.batches:
			takeBatch(rs)
		case s := <-g.raw:
			takeRaw(s)
		case <-flush.C:
			if err := submitAll(); err != nil {
				g.l.Error("submit failed", zap.Error(err))
			}
		case <-epoch.C:
			if err := submitAll(); err != nil {
				g.l.Error("submit failed", zap.Error(err))
			}
			if err := g.publish(); err != nil {
				g.l.Error("snapshot failed", zap.Error(err))
			}
		}
	}
}

// publish merges the devices into the first one and renders its series into the
// AdvancedRegistry vectors with the reference's names, types, Help texts and labels
// (forward.go:18-26, drops.go:18-23, tcpflags.go:18-24, tcpretrans.go:18-24 -- GaugeVec;
// dns.go:21-30,50-66 -- CounterVec), then retires the slots of deleted pods.
// WriteExposition writes the engine's series to w in the Prometheus text exposition
// format (what the AdvancedRegistry's /metrics handler would serve for them), straight from
// the library's rendering (gpuagg_result_text: no copy into Go memory).  A /metrics
// handler for very high cardinalities can serve this instead of walking every series
// into the GaugeVec/CounterVec objects (publish).
func (g *gpuAgg) WriteExposition(w io.Writer) error {
	g.mu.Lock()
	defer g.mu.Unlock()
	if g.stopping || len(g.devs) == 0 {
		return nil
	}
	if len(g.devs) > 1 {
		ctxs := make([]*C.gpuagg_ctx, len(g.devs))
		for i, d := range g.devs {
			ctxs[i] = d.ctx
		}
		if err := check(ctxs[0], C.gpuagg_merge(&ctxs[0], C.size_t(len(ctxs))), "gpuagg_merge"); err != nil {
			return err
		}
	}
	ctx := g.devs[0].ctx
	var r *C.gpuagg_result
	if err := check(ctx, C.gpuagg_snapshot(ctx, &r), "gpuagg_snapshot"); err != nil {
		return err
	}
	defer C.gpuagg_result_free(r)
	var text *C.char
	var n C.size_t
	if err := check(ctx, C.gpuagg_result_text(r, &text, &n), "gpuagg_result_text"); err != nil {
		return err
	}
	if n == 0 {
		return nil
	}
	_, err := w.Write(unsafe.Slice((*byte)(unsafe.Pointer(text)), int(n))) // valid until the free above
	return err
}

func (g *gpuAgg) publish() error {
	g.mu.Lock()
	defer g.mu.Unlock()
	if g.stopping || len(g.devs) == 0 {
		return nil
	}
	if len(g.devs) > 1 {
		ctxs := make([]*C.gpuagg_ctx, len(g.devs))
		for i, d := range g.devs {
			ctxs[i] = d.ctx
		}
		if err := check(ctxs[0], C.gpuagg_merge(&ctxs[0], C.size_t(len(ctxs))), "gpuagg_merge"); err != nil {
			return err
		}
	}
	ctx := g.devs[0].ctx
	var r *C.gpuagg_result
	if err := check(ctx, C.gpuagg_snapshot(ctx, &r), "gpuagg_snapshot"); err != nil {
		return err
	}
	defer C.gpuagg_result_free(r)
	if lost := uint64(C.gpuagg_result_dropped(r)); lost > 0 {
		g.l.Warn("group-by table full: series undercount", zap.Uint64("lost_updates", lost))
	}
	n := int(C.gpuagg_result_count(r))
	// counter series of this snapshot: what was already added per label tuple.  Tuples
	// missing from the snapshot are dropped (their slots were retired), and a value below
	// the last one means the engine restarted the series (a retired slot reused by a pod
	// of the same namespace/name): the whole value is new.
	ctrNext := make(map[string]float64, len(g.ctrLast))
	for i := 0; i < n; i++ {
		var metric, typ, help *C.char
		var nl C.uint32_t
		var names, values **C.char
		var v C.uint64_t
		C.gpuagg_result_series(r, C.size_t(i), &metric, &nl, &names, &values, &v)
		C.gpuagg_result_family(r, C.size_t(i), &typ, &help)
		ns := unsafe.Slice(names, int(nl))
		vs := unsafe.Slice(values, int(nl))
		labels := make([]string, int(nl))
		lvals := make([]string, int(nl))
		for j := range labels {
			labels[j], lvals[j] = C.GoString(ns[j]), C.GoString(vs[j])
		}
		full := C.GoString(metric) // "networkobservability_<name>"
		short := full[len(exporter.RetinaNamespace)+1:]
		if C.GoString(typ) == "counter" {
			vec, ok := g.ctrs[full]
			if !ok {
				vec = exporter.CreatePrometheusCounterVecForMetric(exporter.AdvancedRegistry, short, C.GoString(help), labels...)
				g.ctrs[full] = vec
			}
			// the engine's values are cumulative since reconcile: add the increment
			key := full + "\x00" + strings.Join(lvals, "\x00")
			last, seen := g.ctrLast[key]
			d := float64(v) - last
			if !seen || float64(v) < last {
				d = float64(v)
			}
			if d > 0 {
				vec.WithLabelValues(lvals...).Add(d)
			}
			ctrNext[key] = float64(v)
			continue
		}
		vec, ok := g.vecs[full]
		if !ok {
			vec = exporter.CreatePrometheusGaugeVecForMetric(exporter.AdvancedRegistry, short, C.GoString(help), labels...)
			g.vecs[full] = vec
		}
		vec.WithLabelValues(lvals...).Set(float64(v))
	}
	g.ctrLast = ctrNext
	if g.latency != nil || g.noResponse != nil {
		var st C.gpuagg_latency_state
		if err := check(ctx, C.gpuagg_latency_read(ctx, &st), "gpuagg_latency_read"); err != nil {
			return err
		}
		if g.latency != nil {
			g.latency.mu.Lock()
			g.latency.st = st
			g.latency.mu.Unlock()
		}
		if g.noResponse != nil {
			if d := float64(st.no_response) - g.noRespLast; d > 0 {
				g.noResponse.WithLabelValues("no_response").Add(d)
				g.noRespLast = float64(st.no_response)
			}
		}
	}
	// the epoch is published: DNS ids no series references any more (at this publish and
	// the previous one) are retired, and slots no IP maps to any more are freed (their
	// series keep the last published value, as the reference's gauges of a deleted pod do)
	if err := g.retireDNSLocked(); err != nil {
		return err
	}
	return g.each("gpuagg_retire_slots", func(c *C.gpuagg_ctx) C.int { return C.gpuagg_retire_slots(c, nil) })
}

// retireDNSLocked retires, on every device at once, the dns_ids no group-by key has
// referenced at this call and the previous one (gpuagg_dns_retire's two phases), drops
// them from dnsByID and hands them to the producer caches, so the dictionary is bounded
// by the live series (as the reference's AdvancedRegistry holds its DNS series) instead
// of growing with every payload ever seen.
func (g *gpuAgg) retireDNSLocked() error {
	if len(g.devs) == 0 || len(g.dnsByID) == 0 {
		return nil
	}
	ctxs := make([]*C.gpuagg_ctx, len(g.devs))
	for i, d := range g.devs {
		ctxs[i] = d.ctx
	}
	// every id in use was handed out by InternDNS, so it is a key of dnsByID
	ids := make([]C.uint32_t, len(g.dnsByID))
	var n C.size_t
	if err := check(ctxs[0], C.gpuagg_dns_retire(&ctxs[0], C.size_t(len(ctxs)), &ids[0], C.size_t(len(ids)), &n),
		"gpuagg_dns_retire"); err != nil {
		return err
	}
	if int(n) > len(ids) {
		n = C.size_t(len(ids))
	}
	if n == 0 {
		return nil
	}
	dead := make([]uint32, int(n))
	for i := range dead {
		dead[i] = uint32(ids[i])
		delete(g.dnsByID, dead[i])
	}
	for _, h := range g.dnsRetired {
		h(dead)
	}
	return nil
}

// onDNSRetire registers a producer cache to drop retired dns_ids from.
func (g *gpuAgg) onDNSRetire(h func([]uint32)) {
	g.mu.Lock()
	defer g.mu.Unlock()
	g.dnsRetired = append(g.dnsRetired, h)
}

// Stop stops Start (it waits for it) and releases the contexts.
func (g *gpuAgg) Stop() error {
	g.mu.Lock()
	g.stopping = true
	done := g.done
	g.mu.Unlock()
	if done != nil {
		select { // Start returns once its ctx is cancelled by the manager
		case <-done:
		case <-time.After(10 * time.Second):
			return errors.New("gpuagg: Start did not return; contexts kept")
		}
	}
	g.mu.Lock()
	defer g.mu.Unlock()
	g.destroyLocked()
	return nil
}

func (g *gpuAgg) destroyLocked() {
	for kind, f := range g.feeds {
		C.gpuagg_raw_feed_destroy(f) // before the contexts: it frees their pinned staging
		delete(g.feeds, kind)
	}
	if g.recFeed != nil {
		C.gpuagg_raw_feed_destroy(g.recFeed)
		g.recFeed = nil
	}
	for _, d := range g.devs {
		C.gpuagg_destroy(d.ctx) // frees the pinned batch too
	}
	g.devs = nil
	g.done = nil
}

// ---- the IP cache ---------------------------------------------------------------------

// InternDNS returns the dns_id a DNS producer writes for an AddDNSInfo payload
// (flow_utils.go:186-220), the same on every device.
func (g *gpuAgg) InternDNS(rcode uint32, qtypes []string, query string, ips []string, numAnswers uint32) (uint32, error) {
	g.mu.Lock()
	defer g.mu.Unlock()
	qt, q, ip := C.CString(strings.Join(qtypes, ",")), C.CString(query), C.CString(strings.Join(ips, ","))
	defer C.free(unsafe.Pointer(qt))
	defer C.free(unsafe.Pointer(q))
	defer C.free(unsafe.Pointer(ip))
	var id C.uint32_t
	err := g.each("gpuagg_dns_intern", func(ctx *C.gpuagg_ctx) C.int {
		return C.gpuagg_dns_intern(ctx, C.uint32_t(rcode), qt, q, ip, C.uint32_t(numAnswers), &id)
	})
	if err == nil {
		if g.dnsByID == nil {
			g.dnsByID = make(map[uint32]dnsPayload)
		}
		g.dnsByID[uint32(id)] = dnsPayload{rcode, qtypes, query, ips, numAnswers}
	}
	return uint32(id), err
}

// commitLocked installs the cache's IP -> pod map before a batch that follows a cache
// change (versioned: earlier batches keep the previous map).
func (g *gpuAgg) commitLocked() error {
	if !g.dirty {
		return nil
	}
	g.version++
	v := C.uint64_t(g.version)
	g.dirty = false
	return g.each("gpuagg_cache_commit", func(ctx *C.gpuagg_ctx) C.int { return C.gpuagg_cache_commit(ctx, v) })
}

// ipv4LE is net.ParseIP(s).To4() read little-endian -- the record encoding
// (include/gpuagg.h), the inverse of utils.Int2ip (utils_linux.go:51-55) -- without the
// allocation on the common form: a dotted quad of 1-3 digit decimal octets <= 255 with no
// leading zeros (net.ParseIP rejects those since Go 1.17).  Anything else (IPv4-mapped
// IPv6 text, malformed input) takes net.ParseIP itself, so the result is always exactly
// net.ParseIP's (tests/test_enricher_inverse.py checks a transcription of both paths).
func ipv4LE(s string) (uint32, bool) {
	var v, oct, digits uint32
	dots := uint32(0)
	for i := 0; i < len(s); i++ {
		c := s[i]
		switch {
		case c >= '0' && c <= '9':
			if digits > 0 && oct == 0 { // a leading zero
				return ipv4LESlow(s)
			}
			oct = oct*10 + uint32(c-'0')
			digits++
			if digits > 3 || oct > 255 {
				return ipv4LESlow(s)
			}
		case c == '.':
			if digits == 0 || dots == 3 {
				return ipv4LESlow(s)
			}
			v |= oct << (8 * dots)
			dots++
			oct, digits = 0, 0
		default:
			return ipv4LESlow(s)
		}
	}
	if dots != 3 || digits == 0 {
		return ipv4LESlow(s)
	}
	return v | oct<<24, true
}

func ipv4LESlow(s string) (uint32, bool) {
	p := net.ParseIP(s).To4()
	if p == nil {
		return 0, false
	}
	return binary.LittleEndian.Uint32(p), true
}

func b2u(b bool) uint32 {
	if b {
		return 1
	}
	return 0
}

// PacketRecord is the record of one packetparser event -- the fields of
// packetparserPacket (packetparser_bpfel_x86.go:45-70) as processRecord turns them into a
// flow (packetparser_linux.go:571-631: ToFlow with FORWARDED, HostToNetShort ports,
// ktime.MonotonicOffset added to T_nsec, IsReply, TrafficDirection, TCP flags, TCP id) --
// with exactly the columns packet_decode_kernel produces from the raw sample
// (gpuagg_decode.hip).  Producers that decode themselves call
// gpuAgg.Write(gpuagg.PacketRecord(...)) instead of building a *flow.Flow.
func PacketRecord(tNsec uint64, bytes, srcIP, dstIP uint32, srcPort, dstPort uint16, tsval, tsecr uint32,
	obsPoint, trafficDirection, proto, flags uint8, isReply bool) Record {
	verdict := uint32(flow.Verdict_FORWARDED)
	if trafficDirection > 3 { // not encodable in the meta word: no metric consumes the row
		verdict = 255
	}
	tcpFlags := uint32(0)
	if proto == 6 {
		tcpFlags = uint32(flags) & 0x3f
	}
	obs := uint32(obsPoint)
	if obs > 3 {
		obs = 0
	}
	r := Record{
		SrcIP: srcIP, DstIP: dstIP, Bytes: bytes,
		Meta: uint32(proto) | verdict<<8 | uint32(trafficDirection&3)<<16 | tcpFlags<<21 | b2u(isReply)<<27 |
			obs<<30,
		Ports:  uint32(bits.ReverseBytes16(srcPort)) | uint32(bits.ReverseBytes16(dstPort))<<16,
		DNSID:  0xffffffff,
		TimeNs: uint64(ktime.MonotonicOffset.Nanoseconds() + int64(tNsec)),
	}
	switch obsPoint { // TO_NETWORK carries the request's TSval, FROM_NETWORK the reply's TSecr
	case 3:
		r.TcpID = tsval
	case 2:
		r.TcpID = tsecr
	}
	return r
}

// DropRecord is the record of one dropreason event (dropreason's kernel struct,
// drop_reason.c:39-54, as processRecord builds its flow, dropreason_linux.go:345-386:
// DROPPED, observation point FROM_NETWORK = INGRESS, DropReason = dropType, Bytes =
// skbLen), the columns drop_decode_kernel produces.
func DropRecord(tNsec uint64, srcIP, dstIP uint32, srcPort, dstPort uint16, skbLen uint32, dropType uint16,
	proto uint8) Record {
	verdict := uint32(flow.Verdict_DROPPED)
	if dropType > 7 {
		verdict = 255
	}
	return Record{
		SrcIP: srcIP, DstIP: dstIP, Bytes: skbLen,
		Meta:   uint32(proto) | verdict<<8 | 1<<16 | uint32(dropType&7)<<18 | 2<<30,
		Ports:  uint32(bits.ReverseBytes16(srcPort)) | uint32(bits.ReverseBytes16(dstPort))<<16,
		DNSID:  0xffffffff,
		TimeNs: uint64(ktime.MonotonicOffset.Nanoseconds() + int64(tNsec)),
	}
}

// CacheTee is a cache.CacheInterface that forwards to the agent's cache and mirrors
// every update and delete into the engine, so the GPU's IP table follows exactly the
// reference's cache (cache.go:196-420).  cmd/standard/daemon.go wraps the cache it
// hands to the controllers: `controllerCache = gpuagg.NewCacheTee(controllerCache)`.
type CacheTee struct {
	cache.CacheInterface
}

func NewCacheTee(c cache.CacheInterface) *CacheTee { return &CacheTee{CacheInterface: c} }

func withEngine(fn func(g *gpuAgg) error) error {
	g := Instance()
	if g == nil {
		return nil
	}
	g.mu.Lock()
	defer g.mu.Unlock()
	if len(g.devs) == 0 {
		return nil
	}
	err := fn(g)
	g.dirty = true
	return err
}

func (t *CacheTee) UpdateRetinaEndpoint(ep *common.RetinaEndpoint) error {
	if err := t.CacheInterface.UpdateRetinaEndpoint(ep); err != nil {
		return err
	}
	ips, err := ep.IPs()
	if err != nil {
		return err
	}
	var v4 []uint32
	for _, s := range ips {
		if x, ok := ipv4LE(s); ok {
			v4 = append(v4, x)
		}
	}
	if len(v4) == 0 {
		return nil
	}
	return withEngine(func(g *gpuAgg) error {
		ns, pod := C.CString(ep.Namespace()), C.CString(ep.Name())
		defer C.free(unsafe.Pointer(ns))
		defer C.free(unsafe.Pointer(pod))
		var kind, wname *C.char // getWorkloads: the first owner reference (enricher.go:169-183)
		if refs := ep.OwnerRefs(); len(refs) > 0 && refs[0] != nil {
			kind, wname = C.CString(refs[0].Kind), C.CString(refs[0].Name)
			defer C.free(unsafe.Pointer(kind))
			defer C.free(unsafe.Pointer(wname))
		}
		if err := g.each("gpuagg_cache_update_endpoint", func(ctx *C.gpuagg_ctx) C.int {
			return C.gpuagg_cache_update_endpoint(ctx, ns, pod, kind, wname, (*C.uint32_t)(unsafe.Pointer(&v4[0])), C.size_t(len(v4)))
		}); err != nil {
			return err
		}
		// the slot the update interned (same identity -> same slot), for emitted flows
		var slot C.int32_t
		if err := check(g.devs[0].ctx, C.gpuagg_slot_intern(g.devs[0].ctx, ns, pod, kind, wname, &slot),
			"gpuagg_slot_intern"); err != nil {
			return err
		}
		if g.slotEP == nil {
			g.slotEP = make(map[int32]*common.RetinaEndpoint)
		}
		g.slotEP[int32(slot)] = ep
		return nil
	})
}

func (t *CacheTee) DeleteRetinaEndpoint(epKey string) error {
	if err := t.CacheInterface.DeleteRetinaEndpoint(epKey); err != nil {
		return err
	}
	nsName := strings.SplitN(epKey, "/", 2)
	if len(nsName) != 2 {
		return nil
	}
	return withEngine(func(g *gpuAgg) error {
		ns, pod := C.CString(nsName[0]), C.CString(nsName[1])
		defer C.free(unsafe.Pointer(ns))
		defer C.free(unsafe.Pointer(pod))
		return g.each("gpuagg_cache_delete_endpoint", func(ctx *C.gpuagg_ctx) C.int {
			return C.gpuagg_cache_delete_endpoint(ctx, ns, pod)
		})
	})
}

func (t *CacheTee) UpdateRetinaSvc(svc *common.RetinaSvc) error {
	if err := t.CacheInterface.UpdateRetinaSvc(svc); err != nil {
		return err
	}
	ip, err := svc.GetPrimaryIP()
	if err != nil {
		return err
	}
	x, ok := ipv4LE(ip)
	if !ok {
		return nil
	}
	return withEngine(func(g *gpuAgg) error {
		ns, n := C.CString(svc.Namespace()), C.CString(svc.Name())
		defer C.free(unsafe.Pointer(ns))
		defer C.free(unsafe.Pointer(n))
		return g.each("gpuagg_cache_update_service", func(ctx *C.gpuagg_ctx) C.int {
			return C.gpuagg_cache_update_service(ctx, ns, n, C.uint32_t(x))
		})
	})
}

func (t *CacheTee) DeleteRetinaSvc(svcKey string) error {
	if err := t.CacheInterface.DeleteRetinaSvc(svcKey); err != nil {
		return err
	}
	nsName := strings.SplitN(svcKey, "/", 2)
	if len(nsName) != 2 {
		return nil
	}
	return withEngine(func(g *gpuAgg) error {
		ns, n := C.CString(nsName[0]), C.CString(nsName[1])
		defer C.free(unsafe.Pointer(ns))
		defer C.free(unsafe.Pointer(n))
		return g.each("gpuagg_cache_delete_service", func(ctx *C.gpuagg_ctx) C.int {
			return C.gpuagg_cache_delete_service(ctx, ns, n)
		})
	})
}

func (t *CacheTee) UpdateRetinaNode(node *common.RetinaNode) error {
	if err := t.CacheInterface.UpdateRetinaNode(node); err != nil {
		return err
	}
	x, ok := ipv4LE(node.IPString())
	if !ok {
		return nil
	}
	return withEngine(func(g *gpuAgg) error {
		n := C.CString(node.Name())
		defer C.free(unsafe.Pointer(n))
		return g.each("gpuagg_cache_update_node", func(ctx *C.gpuagg_ctx) C.int {
			return C.gpuagg_cache_update_node(ctx, n, C.uint32_t(x))
		})
	})
}

func (t *CacheTee) DeleteRetinaNode(nodeName string) error {
	if err := t.CacheInterface.DeleteRetinaNode(nodeName); err != nil {
		return err
	}
	return withEngine(func(g *gpuAgg) error {
		n := C.CString(nodeName)
		defer C.free(unsafe.Pointer(n))
		return g.each("gpuagg_cache_delete_node", func(ctx *C.gpuagg_ctx) C.int {
			return C.gpuagg_cache_delete_node(ctx, n)
		})
	})
}
