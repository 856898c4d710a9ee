"""Oracle replay of latency records (tests only)."""

from oracle import latency as L
from oracle import oracle as O
from oracle import records as R


def oracle_latency(recs, api_ips, names=(L.LATENCY, L.HANDSHAKE, L.NO_RESPONSE), batches=None, limit=L.LIMIT):
    m = L.LatencyMetrics(set(names), limit=limit)
    m.add_ips([O.int2ip(int(x)) for x in api_ips])
    for i in range(len(recs.src_ip)):
        f = R.flow_from_record(int(recs.src_ip[i]), int(recs.dst_ip[i]), int(recs.bytes[i]), int(recs.meta[i]),
                               int(recs.ports[i]), 0, {}, int(recs.tcp_id[i]), int(recs.time_ns[i]))
        m.process_flow(f)
    return m


def as_state(m, capacity: bool = False):
    """The oracle's state in gpuagg_latency_state form."""
    def h(x):
        return ([0] * 11, 0, 0) if x is None else (list(x.buckets), x.count, int(x.total))
    lb, lc, ls = h(m.latency)
    hb, hc, hs = h(m.handshake)
    return {"latency_buckets": lb, "latency_count": lc, "latency_sum": ls, "handshake_buckets": hb,
            "handshake_count": hc, "handshake_sum": hs, "no_response": m.no_response or 0,
            "pending": len(m.cache), **({"capacity_evictions": m.capacity_evictions, "peak_live": m.peak_live}
                                       if capacity else {})}
