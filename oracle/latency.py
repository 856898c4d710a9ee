"""Node-apiserver latency metrics, restated (TEST INFRASTRUCTURE ONLY).

Follows pkg/module/metrics/latency.go of the reference:
  * NewLatencyMetrics / Init (:73-150): three metrics, selected by name
    `node_apiserver_latency` (histogram adv_node_apiserver_latency),
    `node_apiserver_handshake_latency` (histogram adv_node_apiserver_tcp_handshake_latency),
    `node_apiserver_no_response` (counter vec adv_node_apiserver_no_response, label
    "no_response"); histograms use prometheus.LinearBuckets(0, 0.5, 10) (:35-39);
  * ProcessFlow (:178-201): TCP with a non-zero TCP id (utils.GetTCPID, flow_utils.go:176-183)
    whose source or destination IP is an apiserver IP;
  * calculateLatency (:256-305): TO_NETWORK packets insert {src, dst, sport, dport, id} ->
    (Time.Nanos, flags) unless present; FROM_NETWORK packets look up the mirrored key,
    observe round((Nanos - t) / 1e6) ms, observe the handshake latency when the stored
    packet had SYN and this one SYN+ACK, and delete the entry;
  * the ttlcache (:118-132): TTL 500 ms, an entry that expires unanswered counts one
    no_response (EvictionReasonExpired); deletions do not count;
  * the cache is github.com/jellydator/ttlcache/v3 v3.3.0 (go.mod:306; not vendored in the
    reference, so its published behaviour is restated here -- parity unpinned, the
    reference's tests never fill the cache): `Get` of a live key "touches" it (its
    expiry becomes now + TTL and it moves to the front of the LRU list, unless
    WithDisableTouchOnHit, which latency.go does not set), so a repeated TO_NETWORK packet
    (same TSval) keeps its request alive; `WithCapacity(LIMIT)` makes `Set` of a new key
    with LIMIT live entries first evict the LRU back (EvictionReasonCapacityReached: no
    no_response).  Every touch happens at the current clock, so LRU order is expiry order.

The reference's TTL clock is the agent's wall clock; a batch replay has none, so this
restatement uses the record timestamps as the clock: before a record is processed every
entry whose expiry (insert clock + 500 ms) lies before the running maximum of the record
times seen so far is evicted (and counted).  The ttlcache capacity (LIMIT = 100000 live
entries, capacity evictions do not count) is enforced: a new request that finds LIMIT
live entries evicts the least recently touched one (`capacity_evictions` counts them).
The latency arithmetic (Nanos only, so a pair that straddles a second boundary gives a
negative latency) is the reference's.
"""

from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field
from decimal import ROUND_HALF_UP, Decimal
from typing import Dict, List, Optional, Set, Tuple

from . import oracle as O

TTL_NS = 500_000_000        # latency.go:34
LIMIT = 100_000             # latency.go:35
BUCKETS = [0.5 * i for i in range(10)]  # LinearBuckets(start 0, width 0.5, count 10)

LATENCY = "node_apiserver_latency"
HANDSHAKE = "node_apiserver_handshake_latency"  # utils/metric_names.go:29
NO_RESPONSE = "node_apiserver_no_response"
FAMILY = {
    LATENCY: ("networkobservability_adv_node_apiserver_latency", "Latency of node apiserver in ms"),
    HANDSHAKE: ("networkobservability_adv_node_apiserver_tcp_handshake_latency",
                "Latency of node apiserver tcp handshake in ms"),
    NO_RESPONSE: ("networkobservability_adv_node_apiserver_no_response",
                  "Number of packets that did not get a response from node apiserver"),
}


def go_round(x: float) -> float:
    """math.Round: half away from zero."""
    d = Decimal(repr(x)).quantize(Decimal(1), rounding=ROUND_HALF_UP)
    return float(d)


@dataclass
class Histogram:
    """prometheus Histogram with upper bounds BUCKETS (+Inf implicit)."""
    buckets: List[int] = field(default_factory=lambda: [0] * (len(BUCKETS) + 1))
    count: int = 0
    total: float = 0.0

    def observe(self, v: float) -> None:
        i = 0
        while i < len(BUCKETS) and v > BUCKETS[i]:
            i += 1
        self.buckets[i] += 1  # non-cumulative; exposition accumulates
        self.count += 1
        self.total += v


@dataclass
class _Entry:
    nanos: int
    syn: bool
    expires: int


class LatencyMetrics:
    def __init__(self, metric_names: Set[str], limit: int = LIMIT):
        self.latency = Histogram() if LATENCY in metric_names else None
        self.handshake = Histogram() if HANDSHAKE in metric_names else None
        self.no_response: Optional[int] = 0 if NO_RESPONSE in metric_names else None
        self.apiserver_ips: Set[str] = set()
        self.cache: "OrderedDict[Tuple, _Entry]" = OrderedDict()
        self.clock = 0
        self.peak_live = 0
        self.limit = limit
        self.capacity_evictions = 0

    # apiserverWatcherCallbackFn (:307-333)
    def add_ips(self, ips: List[str]) -> None:
        self.apiserver_ips.update(ips)

    def remove_ips(self, ips: List[str]) -> None:
        for ip in ips:
            self.apiserver_ips.discard(ip)

    def _expire(self) -> None:
        # touch clocks never decrease, so the LRU order of the OrderedDict (front = least
        # recently touched) is expiry order
        while self.cache:
            k, e = next(iter(self.cache.items()))
            if not self.clock > e.expires:
                break
            del self.cache[k]
            if self.no_response is not None:
                self.no_response += 1

    def process_flow(self, f: O.Flow) -> None:
        if f is None:
            return
        # every record the module sees advances the clock (the cleaner runs regardless)
        self.clock = max(self.clock, f.time_ns)
        self._expire()
        if f.l4 is None or f.l4.proto != "TCP" or f.ip is None:
            return
        tcp_id = f.extensions.tcp_id if f.extensions is not None else 0
        if tcp_id == 0:
            return
        if f.ip.source in self.apiserver_ips or f.ip.destination in self.apiserver_ips:
            self._calculate(f, tcp_id)

    def _calculate(self, f: O.Flow, tcp_id: int) -> None:
        nanos = f.time_ns % 1_000_000_000
        flags = f.l4.flags
        if f.trace_observation_point == O.OBS_TO_NETWORK:
            k = (f.ip.source, f.ip.destination, f.l4.source_port, f.l4.destination_port, tcp_id)
            e = self.cache.get(k)
            if e is not None:  # Get hit: touched (expiry extended, moved to the LRU front)
                e.expires = self.clock + TTL_NS
                self.cache.move_to_end(k)
            else:
                if len(self.cache) >= self.limit:  # Set at capacity: the LRU back goes, uncounted
                    self.cache.popitem(last=False)
                    self.capacity_evictions += 1
                self.cache[k] = _Entry(nanos, bool(flags is not None and flags.SYN), self.clock + TTL_NS)
                self.peak_live = max(self.peak_live, len(self.cache))
        elif f.trace_observation_point == O.OBS_FROM_NETWORK:
            k = (f.ip.destination, f.ip.source, f.l4.destination_port, f.l4.source_port, tcp_id)
            e = self.cache.get(k)
            if e is not None:
                lat = go_round((nanos - e.nanos) / 1_000_000.0)
                if self.latency is not None:
                    self.latency.observe(lat)
                if (self.handshake is not None and e.syn and flags is not None and flags.SYN
                        and flags.ACK):
                    self.handshake.observe(lat)
                del self.cache[k]

    def finish(self, now_ns: int = 0) -> None:
        """Evicts what has expired by the last record time, or by now_ns if later (the
        cleaner goroutine)."""
        self.clock = max(self.clock, now_ns)
        self._expire()

    def state(self) -> Dict[str, object]:
        return {"latency": self.latency, "handshake": self.handshake,
                "no_response": self.no_response, "pending": len(self.cache)}


def render(m: LatencyMetrics) -> str:
    """Prometheus text exposition of the three families (same layout rules as
    oracle/exposition.py; histogram buckets cumulative with le labels, _sum, _count)."""
    from .exposition import go_format_float
    out = []
    fams = []
    if m.latency is not None:
        fams.append((FAMILY[LATENCY][0], FAMILY[LATENCY][1], "histogram", m.latency))
    if m.handshake is not None:
        fams.append((FAMILY[HANDSHAKE][0], FAMILY[HANDSHAKE][1], "histogram", m.handshake))
    if m.no_response:  # the vec child exists from its first Inc (WithLabelValues, :126-129)
        fams.append((FAMILY[NO_RESPONSE][0], FAMILY[NO_RESPONSE][1], "counter", m.no_response))
    for name, help_, typ, v in sorted(fams):
        out.append("# HELP %s %s\n# TYPE %s %s\n" % (name, help_, name, typ))
        if typ == "counter":
            out.append('%s{no_response="no_response"} %s\n' % (name, go_format_float(float(v))))
            continue
        acc = 0
        for ub, c in zip(BUCKETS + [float("inf")], v.buckets):
            acc += c
            le = "+Inf" if ub == float("inf") else go_format_float(ub)
            out.append('%s_bucket{le="%s"} %d\n' % (name, le, acc))
        out.append("%s_sum %s\n%s_count %d\n" % (name, go_format_float(v.total), name, v.count))
    return "".join(out)
