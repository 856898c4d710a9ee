"""Oracle side of the SoA record contract (TEST INFRASTRUCTURE ONLY).

Restates how a decoded flow record -- laid out as the column batch that
``include/gpuagg.h`` documents -- becomes the ``flow.Flow`` each Retina producer
would have built, then replays it through ``oracle.enrich`` and ``oracle.Module``
one flow at a time (lossless replay).

Producers restated:
* packetparser (verdict FORWARDED): packetparser_linux.go:571-631
* dropreason (verdict DROPPED, obs 2 -> INGRESS, no TCP flags): dropreason_linux.go:345-386
* tcpretrans (verdict 15, obs 0 -> EGRESS, TCP flags): tcpretrans_linux.go:124-139
* dns (verdict 16, obs 2/3): dns_linux.go:115-141, flow_utils.go:186-220
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import oracle as O

# meta word layout (restated from DESIGN.md section 3; independent of the product header)
META_PROTO_SHIFT, META_VERDICT_SHIFT, META_TDIR_SHIFT = 0, 8, 16
META_REASON_SHIFT, META_FLAGS_SHIFT, META_REPLY_SHIFT, META_DNSTYPE_SHIFT = 18, 21, 27, 28
META_OBS_SHIFT = 30  # observation point 0-3 (include/gpuagg.h)


def pack_meta(proto: int, verdict: int, tdir: int = 0, reason: int = 0, flags: int = 0,
              is_reply: int = 0, dns_type: int = 0) -> int:
    return ((proto & 0xFF) | ((verdict & 0xFF) << 8) | ((tdir & 3) << 16) | ((reason & 7) << 18)
            | ((flags & 0x3F) << 21) | ((is_reply & 1) << 27) | ((dns_type & 3) << 28))


def pack_meta_np(proto, verdict, tdir=0, reason=0, flags=0, is_reply=0, dns_type=0, obs=0) -> np.ndarray:
    """pack_meta over numpy arrays (fields masked to their widths; an observation point
    above 3 is written as 0, include/gpuagg.h)."""
    u = np.uint32

    def f(x, mask, shift):
        return (np.asarray(x).astype(u) & u(mask)) << u(shift)
    obs = np.asarray(obs).astype(u)
    return (f(proto, 0xFF, META_PROTO_SHIFT) | f(verdict, 0xFF, META_VERDICT_SHIFT)
            | f(tdir, 3, META_TDIR_SHIFT) | f(reason, 7, META_REASON_SHIFT)
            | f(flags, 0x3F, META_FLAGS_SHIFT) | f(is_reply, 1, META_REPLY_SHIFT)
            | f(dns_type, 3, META_DNSTYPE_SHIFT) | f(np.where(obs <= 3, obs, u(0)), 3, META_OBS_SHIFT))


@dataclass
class DnsEntry:
    """One DNS label payload as the producer saw it (dns_linux.go:138)."""
    rcode: int
    qtypes: List[str]
    query: str
    ips: List[str]
    num_answers: int


@dataclass
class Batch:
    """Column batch, numpy uint32 arrays of equal length."""
    src_ip: np.ndarray
    dst_ip: np.ndarray
    bytes: np.ndarray
    meta: np.ndarray
    ports: Optional[np.ndarray] = None
    dns_id: Optional[np.ndarray] = None
    tcp_id: Optional[np.ndarray] = None   # u32 (latency)
    time_ns: Optional[np.ndarray] = None  # u64 (latency)

    def __len__(self) -> int:
        return int(self.src_ip.shape[0])

    def slice(self, a: int, b: int) -> "Batch":
        def s(x):
            return None if x is None else x[a:b]
        return Batch(self.src_ip[a:b], self.dst_ip[a:b], self.bytes[a:b], self.meta[a:b],
                     s(self.ports), s(self.dns_id), s(self.tcp_id), s(self.time_ns))


def flow_from_record(src_ip: int, dst_ip: int, nbytes: int, meta: int, ports: int,
                     dns_id: int, dns_dict: Dict[int, DnsEntry], tcp_id: int = 0,
                     time_ns: int = 0) -> O.Flow:
    proto = meta & 0xFF
    verdict = (meta >> 8) & 0xFF
    tdir = (meta >> 16) & 3
    reason = (meta >> 18) & 7
    flags = (meta >> 21) & 0x3F
    dns_type = (meta >> 28) & 3
    sport, dport = ports & 0xFFFF, (ports >> 16) & 0xFFFF
    obs = (meta >> 30) & 3
    f = O.to_flow(O.int2ip(src_ip), O.int2ip(dst_ip), sport, dport, proto, obs, verdict)
    f.traffic_direction = tdir
    f.time_ns = time_ns
    meta_ext = O.RetinaMetadata(bytes=nbytes, tcp_id=tcp_id)
    verdict = f.verdict  # after ToFlow's 0 -> FORWARDED (flow_utils.go:94-96)
    if verdict in (O.VERDICT_FORWARDED, O.VERDICT_RETRANSMISSION):
        O.add_tcp_flags(f, (flags & 2) >> 1, (flags & 16) >> 4, flags & 1, (flags & 4) >> 2,
                        (flags & 8) >> 3, (flags & 32) >> 5)
    if verdict == O.VERDICT_DROPPED:
        meta_ext.drop_reason = reason
    f.extensions = meta_ext
    if verdict == O.VERDICT_DNS:
        e = dns_dict[dns_id]
        qr = {O.DNS_TYPE_QUERY: "Q", O.DNS_TYPE_RESPONSE: "R"}.get(dns_type, "U")
        O.add_dns_info(f, meta_ext, qr, e.rcode, e.query, e.qtypes, e.num_answers, e.ips)
    return f


@dataclass
class EndpointSpec:
    """A pod as the control plane reports it (RetinaEndpoint subset)."""
    namespace: str
    name: str
    ips: List[int]                       # LE u32 IPv4, primary first
    owner_refs: Optional[List[Tuple[str, str]]] = None  # (kind, name)


def build_cache(endpoints: Sequence[EndpointSpec]) -> O.Cache:
    c = O.Cache()
    for ep in endpoints:
        c.update_retina_endpoint(O.RetinaEndpoint(
            name=ep.name, namespace=ep.namespace, ipv4=O.int2ip(ep.ips[0]),
            other_ipv4s=[O.int2ip(x) for x in ep.ips[1:]],
            owner_refs=None if ep.owner_refs is None else [O.Workload(k, n) for k, n in ep.owner_refs]))
    return c


def replay(batch: Batch, cache: O.Cache, module: O.Module,
           dns_dict: Optional[Dict[int, DnsEntry]] = None) -> None:
    """Lossless replay: every record -> producer flow -> enricher -> every metric."""
    dns_dict = dns_dict or {}
    n = len(batch)
    ports = batch.ports if batch.ports is not None else np.zeros(n, np.uint32)
    dns_id = batch.dns_id if batch.dns_id is not None else np.zeros(n, np.uint32)
    for s, d, b, m, p, q in zip(batch.src_ip.tolist(), batch.dst_ip.tolist(), batch.bytes.tolist(),
                                batch.meta.tolist(), ports.tolist(), dns_id.tolist()):
        f = flow_from_record(s, d, b, m, p, q, dns_dict)
        f = O.enrich(cache, f)
        if f is not None:
            module.process_flow(f)


def spec_from_json(items) -> List[O.MetricsContextOptions]:
    return [O.MetricsContextOptions(i["metric_name"], i.get("source_labels"),
                                    i.get("destination_labels")) for i in items]


def series_to_jsonable(series) -> List[list]:
    """Canonical sorted list [[metric, [[label, value], ...], int], ...]."""
    out = [[k[0], [list(x) for x in k[1]], v] for k, v in series.items()]
    out.sort(key=lambda e: (e[0], e[1]))
    return out
