// Copyright (c) the retina_amd authors.
//
// Package gpuagg is the Retina plugin that drives the MI355X flow-aggregation engine
// through its C ABI (include/gpuagg.h). It keeps the registry.Plugin interface
// (pkg/plugin/registry/registry.go:16-34) so PluginManager can run it like any other
// plugin, and it replaces the enricher + advanced-metrics goroutines
// (pkg/enricher/enricher.go:68-135, pkg/module/metrics/metrics_module.go:276-305).
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
	"fmt"
	"sync"
	"time"
	"unsafe"

	v1 "github.com/cilium/cilium/pkg/hubble/api/v1"
	api "github.com/microsoft/retina/crd/api/v1alpha1"
	kcfg "github.com/microsoft/retina/pkg/config"
	"github.com/microsoft/retina/pkg/exporter"
	"github.com/microsoft/retina/pkg/log"
	"github.com/microsoft/retina/pkg/plugin/registry"
	"github.com/prometheus/client_golang/prometheus"
	"go.uber.org/zap"
)

const (
	name          = "gpuagg"
	batchCapacity = 1 << 20
	flushInterval = 100 * time.Millisecond
	scrapeEpoch   = 5 * time.Second
)

// Record is one decoded flow in the column layout of include/gpuagg.h. Producers
// (packetparser.processRecord, dropReason.processRecord, dns.eventHandler,
// tcpretrans.eventHandler) fill it instead of building a *flow.Flow.
type Record struct {
	SrcIP, DstIP, Bytes, Meta, Ports, DNSID uint32
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

type rawSample struct {
	kind int
	b    []byte
}

type gpuAgg struct {
	cfg *kcfg.Config
	l   *log.ZapLogger

	mu      sync.Mutex
	ctx     *C.gpuagg_ctx
	batch   *C.gpuagg_batch
	n       int
	records chan Record
	raw     chan rawSample
	rawBuf  map[int][]byte // per kind: back-to-back raw records awaiting submit
	vecs    map[string]*prometheus.GaugeVec
}

func init() {
	registry.Add(name, New)
}

// New is the registry.PluginFunc (registry.go:37).
func New(cfg *kcfg.Config) registry.Plugin {
	return &gpuAgg{cfg: cfg, l: log.Logger().Named(name), records: make(chan Record, 1<<16),
		raw: make(chan rawSample, 1<<16), rawBuf: map[int][]byte{}}
}

func (g *gpuAgg) Name() string                           { return name }
func (g *gpuAgg) Generate(ctx context.Context) error     { return nil }
func (g *gpuAgg) Compile(ctx context.Context) error      { return nil }
func (g *gpuAgg) SetupChannel(c chan *v1.Event) error    { return nil } // no Hubble events
func (g *gpuAgg) lastError() string                      { return C.GoString(C.gpuagg_last_error(g.ctx)) }
func check(g *gpuAgg, rc C.int, what string) error {
	if rc != C.GPUAGG_OK {
		return fmt.Errorf("%s: %d: %s", what, int(rc), g.lastError())
	}
	return nil
}

// Init creates the device context (one per GPU; device 0 here).
func (g *gpuAgg) Init() error {
	remote := C.int32_t(0)
	if g.cfg.RemoteContext {
		remote = 1
	}
	cfg := C.gpuagg_config{
		abi_version: C.GPUAGG_ABI_VERSION, device: 0, remote_context: remote,
		max_slots: 1 << 20, max_ips: 1 << 21, sparse_capacity_log2: 24,
	}
	if rc := C.gpuagg_create(&cfg, &g.ctx); rc != C.GPUAGG_OK {
		return fmt.Errorf("gpuagg_create: %d (an MI355X/gfx950 is required)", int(rc))
	}
	return check(g, C.gpuagg_alloc_batch(g.ctx, batchCapacity, &g.batch), "gpuagg_alloc_batch")
}

// Reconcile mirrors Module.Reconcile (metrics_module.go:142-203) for the spec's
// context options.
func (g *gpuAgg) Reconcile(spec *api.MetricsSpec) error {
	g.mu.Lock()
	defer g.mu.Unlock()
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
		view := (*[1 << 20]*C.char)(arr)
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
	exporter.ResetAdvancedMetricsRegistry()
	g.vecs = map[string]*prometheus.GaugeVec{}
	return check(g, C.gpuagg_reconcile(g.ctx, p, C.size_t(len(opts))), "gpuagg_reconcile")
}

// Write is what producers call per decoded record (Enricher.Write's replacement).
func (g *gpuAgg) Write(r Record) { g.records <- r }

// WriteRaw takes one perf RawSample of the given kind; a sample of the wrong size is
// refused like binary.Read's size mismatch (dropreason_linux.go:347-352).
func (g *gpuAgg) WriteRaw(kind int, sample []byte) error {
	if sz, ok := rawSize[kind]; !ok || len(sample) != sz {
		return fmt.Errorf("gpuagg: raw sample of %d bytes for kind %d", len(sample), kind)
	}
	g.raw <- rawSample{kind, sample}
	return nil
}

// Start blocks until ctx is done (PluginManager runs it in an errgroup goroutine,
// pluginmanager.go:166-169).
func (g *gpuAgg) Start(ctx context.Context) error {
	flush := time.NewTicker(flushInterval)
	epoch := time.NewTicker(scrapeEpoch)
	defer flush.Stop()
	defer epoch.Stop()
	cols := g.batch.cols
	col := func(p *C.uint32_t) []uint32 { return unsafe.Slice((*uint32)(unsafe.Pointer(p)), batchCapacity) }
	src, dst, byt, meta, ports, dns := col(cols.src_ip), col(cols.dst_ip), col(cols.bytes), col(cols.meta), col(cols.ports), col(cols.dns_id)
	submit := func() error {
		if g.n == 0 {
			return nil
		}
		g.mu.Lock()
		defer g.mu.Unlock()
		err := check(g, C.gpuagg_submit(g.ctx, g.batch, C.size_t(g.n)), "gpuagg_submit")
		g.n = 0
		return err
	}
	submitRaw := func(kind int) error {
		buf := g.rawBuf[kind]
		if len(buf) == 0 {
			return nil
		}
		g.mu.Lock()
		defer g.mu.Unlock()
		// gpuagg_submit_raw copies the records to HBM before it returns
		err := check(g, C.gpuagg_submit_raw(g.ctx, C.int(kind), unsafe.Pointer(&buf[0]),
			C.size_t(len(buf)/rawSize[kind])), "gpuagg_submit_raw")
		g.rawBuf[kind] = buf[:0]
		return err
	}
	submitAll := func() error {
		err := submit()
		for kind := range rawSize {
			if e := submitRaw(kind); e != nil && err == nil {
				err = e
			}
		}
		return err
	}
	for {
		select {
		case <-ctx.Done():
			return submitAll()
		case r := <-g.records:
			src[g.n], dst[g.n], byt[g.n], meta[g.n], ports[g.n], dns[g.n] = r.SrcIP, r.DstIP, r.Bytes, r.Meta, r.Ports, r.DNSID
			g.n++
			if g.n == batchCapacity {
				if err := submit(); err != nil {
					g.l.Error("submit failed", zap.Error(err))
				}
			}
		case s := <-g.raw:
			g.rawBuf[s.kind] = append(g.rawBuf[s.kind], s.b...)
			if len(g.rawBuf[s.kind]) >= batchCapacity*rawSize[s.kind] {
				if err := submitRaw(s.kind); err != nil {
					g.l.Error("raw submit failed", zap.Error(err))
				}
			}
		case <-flush.C:
			if err := submitAll(); err != nil {
				g.l.Error("submit failed", zap.Error(err))
			}
		case <-epoch.C:
			if err := g.publish(); err != nil {
				g.l.Error("snapshot failed", zap.Error(err))
			}
		}
	}
}

// publish renders the engine's series into the AdvancedRegistry gauge vectors with
// the reference's names and labels (forward.go:100-118, drops.go:268-286, ...).
func (g *gpuAgg) publish() error {
	g.mu.Lock()
	defer g.mu.Unlock()
	var r *C.gpuagg_result
	if err := check(g, C.gpuagg_snapshot(g.ctx, &r), "gpuagg_snapshot"); err != nil {
		return err
	}
	defer C.gpuagg_result_free(r)
	n := int(C.gpuagg_result_count(r))
	for i := 0; i < n; i++ {
		var metric *C.char
		var nl C.uint32_t
		var names, values **C.char
		var v C.uint64_t
		C.gpuagg_result_series(r, C.size_t(i), &metric, &nl, &names, &values, &v)
		ns := unsafe.Slice(names, int(nl))
		vs := unsafe.Slice(values, int(nl))
		labels := make([]string, int(nl))
		lvals := make([]string, int(nl))
		for j := range labels {
			labels[j], lvals[j] = C.GoString(ns[j]), C.GoString(vs[j])
		}
		full := C.GoString(metric) // "networkobservability_<name>"
		vec, ok := g.vecs[full]
		if !ok {
			vec = exporter.CreatePrometheusGaugeVecForMetric(exporter.AdvancedRegistry,
				full[len(exporter.RetinaNamespace)+1:], full, labels...)
			g.vecs[full] = vec
		}
		vec.WithLabelValues(lvals...).Set(float64(v))
	}
	return nil
}

func (g *gpuAgg) Stop() error {
	g.mu.Lock()
	defer g.mu.Unlock()
	if g.ctx != nil {
		C.gpuagg_destroy(g.ctx)
		g.ctx = nil
	}
	return nil
}
