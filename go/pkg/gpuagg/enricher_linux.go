//go:build linux && gpuagg

// Enricher: the engine behind the reference's enricher.EnricherInterface
// (pkg/enricher/types.go:12-16), so unmodified producers -- packetparser
// (packetparser_linux.go:638-640), dropreason (dropreason_linux.go:397-399), dns
// (dns_linux.go:150-152), tcpretrans (tcpretrans_linux.go:148-151) -- keep calling
// Write(*v1.Event) and the metrics module's consumers keep reading ExportReader().
//
// Write turns each flow back into the record utils.ToFlow was built from (flowToRecord:
// the inverse of ToFlow + AddRetinaMetadata / AddTCPFlags / AddDNSInfo / AddDropReason,
// flow_utils.go:33-300) and hands records to the plugin in slices (WriteBatch: one channel
// operation per slice, not per flow).  Enrichment happens on the GPU; the enriched flows
// the engine emits (gpuagg_submit_enrich, SetupChannel's path) are written to an output
// container.Ring as Enricher.export does (enricher.go:137-140), which ExportReader serves.
//
// Wiring (pkg/enricher/enricher.go:New / Instance): where the agent builds the enricher,
//
//	e := gpuagg.NewEnricher(ctx, gpuagg.Instance())
//	e.Run()
//
// and producers take `e` wherever they took enricher.Instance() (their field is already
// typed enricher.EnricherInterface, types_linux.go:116 and dropreason types_linux.go:47).
package gpuagg

import (
	"context"
	"runtime"
	"strconv"
	"strings"
	"sync"
	"time"

	"github.com/cilium/cilium/api/v1/flow"
	v1 "github.com/cilium/cilium/pkg/hubble/api/v1"
	"github.com/cilium/cilium/pkg/hubble/container"
	"github.com/microsoft/retina/pkg/log"
	"github.com/microsoft/retina/pkg/metrics"
	"github.com/microsoft/retina/pkg/utils"
	"go.uber.org/zap"
)

// flows converted per WriteBatch slice
const enricherSlice = 4096

// conversion workers at most (GOMAXPROCS below that)
const enricherMaxWorkers = 16

// Enricher implements enricher.EnricherInterface over the plugin.
//
// The reference enriches on one goroutine (enricher.go:68-99).  Here the per-flow cost is
// the conversion back to a record -- one Any UnmarshalTo of the RetinaMetadata extension,
// two IPv4 parses (ipv4LE: no allocation on dotted quads), the field reads -- so it runs on
// GOMAXPROCS workers (at most enricherMaxWorkers).  Write picks a flow's worker by a hash
// of its direction-free (ip, port) ends and protocol, so a connection's request and reply
// keep their order through one worker (the node-apiserver latency join pairs a request
// with the reply after it); each worker fills its own []Record slice and hands it over
// with one WriteBatch per enricherSlice flows or flushInterval.
type Enricher struct {
	ctx context.Context
	g   *gpuAgg
	l   *log.ZapLogger

	in  []chan *v1.Event // one input channel per conversion worker
	out *container.Ring
	// enriched flows from the engine (the plugin's SetupChannel consumer)
	enriched chan *v1.Event

	dnsMu  sync.RWMutex
	dnsIDs map[string]uint32 // AddDNSInfo payload -> dns_id (gpuagg_dns_intern), cached
	once   sync.Once
}

// NewEnricher returns the engine-backed enricher; g is the registered plugin (Instance()).
func NewEnricher(ctx context.Context, g *gpuAgg) *Enricher {
	w := runtime.GOMAXPROCS(0)
	if w > enricherMaxWorkers {
		w = enricherMaxWorkers
	}
	if w < 1 {
		w = 1
	}
	e := &Enricher{
		ctx: ctx, g: g, l: log.Logger().Named("gpuagg-enricher"),
		in: make([]chan *v1.Event, w), out: container.NewRing(container.Capacity1023),
		enriched: make(chan *v1.Event, channelDepth), dnsIDs: map[string]uint32{},
	}
	for i := range e.in {
		e.in[i] = make(chan *v1.Event, channelDepth)
	}
	g.onDNSRetire(e.dropDNS)
	return e
}

// dropDNS forgets cached payloads whose dns_id the engine retired (gpuagg_dns_retire at a
// publish): the next record with such a payload interns it again.  Called with the
// plugin's lock held; dnsID never holds dnsMu while it takes that lock.
func (e *Enricher) dropDNS(ids []uint32) {
	dead := make(map[uint32]struct{}, len(ids))
	for _, id := range ids {
		dead[id] = struct{}{}
	}
	e.dnsMu.Lock()
	for k, id := range e.dnsIDs {
		if _, ok := dead[id]; ok {
			delete(e.dnsIDs, k)
		}
	}
	e.dnsMu.Unlock()
}

// Run starts the conversion workers and the export loop (enricher.go:69-98 starts one
// goroutine reading the input ring).
func (e *Enricher) Run() {
	e.once.Do(func() {
		if err := e.g.SetupChannel(e.enriched); err != nil {
			e.l.Error("gpuagg enricher: SetupChannel failed; no enriched flows will be exported", zap.Error(err))
		}
		for i := range e.in {
			go e.convert(e.in[i])
		}
		go e.export()
	})
}

// Write never blocks the producer: a full input channel drops the flow and counts it, as
// the reference's ring overwrites its oldest entry (enricher.go:185-187).
func (e *Enricher) Write(ev *v1.Event) {
	w := 0
	if len(e.in) > 1 {
		w = int(flowKey(ev) % uint64(len(e.in)))
	}
	select {
	case e.in[w] <- ev:
	default:
		metrics.LostEventsCounter.WithLabelValues(utils.BufferedChannel, "gpuagg-enricher").Inc()
	}
}

// flowKey is FNV-1a over a flow's direction-free 5-tuple as text: the two (ip, port)
// ends in order, then the protocol.  It reads the strings in place (no parse, no
// allocation); a non-flow event hashes to 0.
func flowKey(ev *v1.Event) uint64 {
	f, ok := ev.GetEvent().(*flow.Flow)
	if !ok || f == nil {
		return 0
	}
	a, b := f.GetIP().GetSource(), f.GetIP().GetDestination()
	var pa, pb, proto uint32
	if tcp := f.GetL4().GetTCP(); tcp != nil {
		pa, pb, proto = tcp.GetSourcePort(), tcp.GetDestinationPort(), 6
	} else if udp := f.GetL4().GetUDP(); udp != nil {
		pa, pb, proto = udp.GetSourcePort(), udp.GetDestinationPort(), 17
	}
	if a > b || (a == b && pa > pb) {
		a, b, pa, pb = b, a, pb, pa
	}
	const prime = 1099511628211
	h := uint64(14695981039346656037)
	for i := 0; i < len(a); i++ {
		h = (h ^ uint64(a[i])) * prime
	}
	h = (h ^ uint64(pa) ^ 0x100000000) * prime
	for i := 0; i < len(b); i++ {
		h = (h ^ uint64(b[i])) * prime
	}
	h = (h ^ uint64(pb) ^ uint64(proto)<<16 ^ 0x200000000) * prime
	return h
}

// ExportReader is enricher.go:189-191: a reader from the oldest write of the output ring.
func (e *Enricher) ExportReader() *container.RingReader {
	return container.NewRingReader(e.out, e.out.OldestWrite())
}

func (e *Enricher) convert(in chan *v1.Event) {
	buf := make([]Record, 0, enricherSlice)
	tick := time.NewTicker(flushInterval)
	defer tick.Stop()
	flush := func() {
		if len(buf) == 0 {
			return
		}
		e.g.WriteBatch(buf) // the slice is the plugin's from here on
		buf = make([]Record, 0, enricherSlice)
	}
	for {
		select {
		case <-e.ctx.Done():
			flush()
			return
		case ev := <-in:
			f, ok := ev.GetEvent().(*flow.Flow)
			if !ok || f == nil {
				continue // enricher.go:86-96: only flows are enriched
			}
			r, ok := e.flowToRecord(f)
			if !ok {
				continue
			}
			buf = append(buf, r)
			if len(buf) == enricherSlice {
				flush()
			}
		case <-tick.C:
			flush()
		}
	}
}

func (e *Enricher) export() {
	for {
		select {
		case <-e.ctx.Done():
			return
		case ev := <-e.enriched:
			e.out.Write(ev)
		}
	}
}

// flowToRecord inverts utils.ToFlow and the metadata helpers: every field a metric reads
// comes back into the record's columns (include/gpuagg.h "Records").  Flows the
// reference's enrich drops before export (enricher.go:102-124: IPv6, an empty source or
// destination IP) are dropped here too.
func (e *Enricher) flowToRecord(f *flow.Flow) (Record, bool) {
	ip := f.GetIP()
	if ip == nil || ip.GetIpVersion() > flow.IPVersion_IPv4 || ip.GetSource() == "" || ip.GetDestination() == "" {
		return Record{}, false
	}
	src, ok1 := ipv4LE(ip.GetSource())
	dst, ok2 := ipv4LE(ip.GetDestination())
	if !ok1 || !ok2 {
		return Record{}, false
	}
	var proto, sport, dport, flags uint32
	if tcp := f.GetL4().GetTCP(); tcp != nil {
		proto, sport, dport = 6, tcp.GetSourcePort(), tcp.GetDestinationPort()
		if fl := tcp.GetFlags(); fl != nil { // bits FIN, SYN, RST, PSH, ACK, URG (types_linux.go:22-31)
			flags = b2u(fl.GetFIN()) | b2u(fl.GetSYN())<<1 | b2u(fl.GetRST())<<2 | b2u(fl.GetPSH())<<3 |
				b2u(fl.GetACK())<<4 | b2u(fl.GetURG())<<5
		}
	} else if udp := f.GetL4().GetUDP(); udp != nil {
		proto, sport, dport = 17, udp.GetSourcePort(), udp.GetDestinationPort()
	}
	meta := &utils.RetinaMetadata{}
	if x := f.GetExtensions(); x != nil {
		_ = x.UnmarshalTo(meta) // as utils.PacketSize / GetTCPID / GetDNS do (errors ignored there too)
	}
	var obs uint32 // the observation point ToFlow received (flow_utils.go:72-92)
	switch f.GetTraceObservationPoint() {
	case flow.TraceObservationPoint_TO_ENDPOINT:
		obs = 1
	case flow.TraceObservationPoint_FROM_NETWORK:
		obs = 2
	case flow.TraceObservationPoint_TO_NETWORK:
		obs = 3
	}
	verdict := uint32(f.GetVerdict()) & 0xff
	// rows the raw decode leaves out as well (PacketRecord / DropRecord: verdict 255, which no
	// metric consumes): a traffic direction the meta word cannot carry, a drop type past
	// the enum
	if uint32(f.GetTrafficDirection()) > 3 || (f.GetVerdict() == flow.Verdict_DROPPED && uint32(meta.GetDropReason()) > 7) {
		verdict = 255
	}
	r := Record{
		SrcIP: src, DstIP: dst, Bytes: meta.GetBytes(),
		Meta: proto | verdict<<8 | (uint32(f.GetTrafficDirection())&3)<<16 | (uint32(meta.GetDropReason())&7)<<18 |
			flags<<21 | b2u(f.GetIsReply().GetValue())<<27 | (uint32(meta.GetDnsType())&3)<<28 | obs<<30,
		Ports: sport | dport<<16, DNSID: 0xffffffff, TcpID: uint32(meta.GetTcpId()),
	}
	if t := f.GetTime(); t != nil {
		r.TimeNs = uint64(t.AsTime().UnixNano())
	}
	if dns := f.GetL7().GetDns(); dns != nil {
		id, err := e.dnsID(dns.GetRcode(), dns.GetQtypes(), dns.GetQuery(), dns.GetIps(), meta.GetNumResponses())
		if err != nil {
			e.l.Warn("gpuagg enricher: DNS payload not interned", zap.Error(err))
			return Record{}, false
		}
		r.DNSID = id
	}
	return r, true
}

func (e *Enricher) dnsID(rcode uint32, qtypes []string, query string, ips []string, n uint32) (uint32, error) {
	key := strings.Join([]string{query, strings.Join(qtypes, ","), strings.Join(ips, ","),
		strconv.FormatUint(uint64(rcode), 10), strconv.FormatUint(uint64(n), 10)}, "\x00")
	e.dnsMu.RLock()
	id, ok := e.dnsIDs[key]
	e.dnsMu.RUnlock()
	if ok {
		return id, nil
	}
	id, err := e.g.InternDNS(rcode, qtypes, query, ips, n)
	if err != nil {
		return 0, err
	}
	e.dnsMu.Lock()
	e.dnsIDs[key] = id
	e.dnsMu.Unlock()
	return id, nil
}
