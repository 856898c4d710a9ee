"""CPU oracle: a plain-Python restatement of Retina's enricher + advanced-metrics path.

TEST INFRASTRUCTURE ONLY. Nothing in the product (``retina_amd/``, ``include/``)
imports, links or executes this module; only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may use it, and only as the checker.

It restates, per flow and in the reference's own structure, the Go code of
matmerr/retina @ 2025-03-28 (paths relative to the reference root):

* ``utils.ToFlow`` / ``AddTCPFlags`` / ``AddDNSInfo`` / ``GetDNS`` /
  ``DNSRcodeToString`` / ``PacketSize`` / ``DropReasonDescription``
  -- pkg/utils/flow_utils.go:33-305
* ``Int2ip`` / ``HostToNetShort`` -- pkg/utils/utils_linux.go:51-70
* packetparser record decode -- pkg/plugin/packetparser/packetparser_linux.go:571-631
* enricher -- pkg/enricher/enricher.go:102-183
* IP cache -- pkg/controllers/cache/cache.go:110-169,204-420; pkg/common/ipaddr.go:35-50
* context options -- pkg/module/metrics/types.go:109-368
* forward / drop / tcpflags / tcpretrans / dns metrics -- pkg/module/metrics/{forward,drops,
  tcpflags,tcpretrans,dns}.go
* metric dispatch -- pkg/module/metrics/metrics_module.go:205-305

Parity status: pinned by the reference's own known-answer tests (transcribed into
``tests/golden/reference_kat.json`` and checked by ``tests/test_oracle_kat.py``).
Enum *names* that come from cilium's flow.proto (TrafficDirection) are not in the
reference tree; they follow from the reference's Go identifiers (flow_utils.go:75-91:
protoc-gen-go's <Enum>_<value name> constants, whose String() is the value name;
reference_kat.json traffic_direction_identifiers).  Prometheus float64 accumulation is replaced by exact
integer sums (identical while < 2**53).
"""

from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

# ---------------------------------------------------------------------------------
# enums
# ---------------------------------------------------------------------------------

# cilium api/v1/flow: Verdict (FORWARDED=1, DROPPED=2); Retina extensions
# pkg/utils/flow_utils.go:19-21.
VERDICT_UNKNOWN = 0
VERDICT_FORWARDED = 1
VERDICT_DROPPED = 2
VERDICT_RETRANSMISSION = 15
VERDICT_DNS = 16

# cilium flow.TrafficDirection: names from the Go identifiers TrafficDirection_<name>
# (pkg/utils/flow_utils.go:75-91); numbers are internal to this restatement.
TRAFFIC_DIRECTION_NAMES = {0: "TRAFFIC_DIRECTION_UNKNOWN", 1: "INGRESS", 2: "EGRESS"}
TD_UNKNOWN, TD_INGRESS, TD_EGRESS = 0, 1, 2

# cilium flow.TraceObservationPoint values used by ToFlow (flow_utils.go:72-92).
OBS_TO_STACK, OBS_TO_ENDPOINT, OBS_FROM_NETWORK, OBS_TO_NETWORK, OBS_UNKNOWN = (
    "TO_STACK", "TO_ENDPOINT", "FROM_NETWORK", "TO_NETWORK", "UNKNOWN_POINT")

# pkg/utils/metadata_linux.pb.go:87-95
DROP_REASON_NAMES = {
    0: "IPTABLE_RULE_DROP",
    1: "IPTABLE_NAT_DROP",
    2: "TCP_CONNECT_BASIC",
    3: "TCP_ACCEPT_BASIC",
    4: "TCP_CLOSE_BASIC",
    5: "CONNTRACK_ADD_DROP",
    6: "UNKNOWN_DROP",
}
# pkg/utils/metadata_linux.pb.go:33-42
DNS_TYPE_UNKNOWN, DNS_TYPE_QUERY, DNS_TYPE_RESPONSE = 0, 1, 2


def enum_string(names: Dict[int, str], v: int) -> str:
    """protobuf-go Enum.String(): the value name, or the decimal number if unnamed."""
    return names.get(v, str(v))


def traffic_direction_string(v: int) -> str:
    return enum_string(TRAFFIC_DIRECTION_NAMES, v)


# pkg/utils/attr_utils.go:67-85
FLAG_SYN, FLAG_SYNACK, FLAG_ACK, FLAG_FIN, FLAG_RST, FLAG_PSH, FLAG_ECE, FLAG_CWR, FLAG_URG = (
    "SYN", "SYNACK", "ACK", "FIN", "RST", "PSH", "ECE", "CWR", "URG")
DNS_REQUEST_LABELS = ["query_type", "query"]
DNS_RESPONSE_LABELS = ["return_code", "query_type", "query", "response", "num_response"]

# pkg/utils/metric_names.go:11-37
DROPPED_PACKETS_GAUGE = "drop_count"
DROP_BYTES_GAUGE = "drop_bytes"
FORWARD_PACKETS_GAUGE = "forward_count"
FORWARD_BYTES_GAUGE = "forward_bytes"
TCP_FLAG_GAUGE = "tcp_flag_gauges"
TCP_RETRANS_COUNT = "tcp_retransmission_count"
DNS_REQUEST_COUNTER = "dns_request_count"
DNS_RESPONSE_COUNTER = "dns_response_count"

RETINA_NAMESPACE = "networkobservability"  # pkg/exporter/prometheusexporter.go:11
APISERVER_ENDPOINT_NAME = "kubernetes-apiserver"  # pkg/common/types.go:15

# ---------------------------------------------------------------------------------
# flow model (subset of cilium flow.Flow that the path reads)
# ---------------------------------------------------------------------------------


@dataclass
class Workload:
    kind: str
    name: str


@dataclass
class Endpoint:
    namespace: str = ""
    pod_name: str = ""
    labels: List[str] = field(default_factory=list)
    workloads: Optional[List[Workload]] = None


@dataclass
class IP:
    source: str = ""
    destination: str = ""
    ip_version: int = 1


@dataclass
class TCPFlags:
    FIN: bool = False
    SYN: bool = False
    RST: bool = False
    PSH: bool = False
    ACK: bool = False
    URG: bool = False
    ECE: bool = False
    CWR: bool = False


@dataclass
class L4:
    proto: str  # "TCP" | "UDP"
    source_port: int = 0
    destination_port: int = 0
    flags: Optional[TCPFlags] = None  # TCP only


@dataclass
class RetinaMetadata:
    bytes: int = 0
    drop_reason: int = 0
    dns_type: int = DNS_TYPE_UNKNOWN
    num_responses: int = 0
    tcp_id: int = 0


@dataclass
class DNS:
    rcode: int = 0
    query: str = ""
    qtypes: List[str] = field(default_factory=list)
    ips: List[str] = field(default_factory=list)


@dataclass
class Flow:
    ip: Optional[IP] = None
    l4: Optional[L4] = None
    verdict: int = VERDICT_UNKNOWN
    traffic_direction: int = TD_UNKNOWN
    trace_observation_point: str = OBS_UNKNOWN
    is_reply: Optional[bool] = False
    source: Optional[Endpoint] = None
    destination: Optional[Endpoint] = None
    extensions: Optional[RetinaMetadata] = None
    dns: Optional[DNS] = None  # flow.L7.Dns
    l7_type: str = ""
    time_ns: int = 0           # ToFlow's ts (decodeTime keeps every nanosecond, flow_utils.go:307-317)


# ---------------------------------------------------------------------------------
# a1 / a2: record decode and ToFlow
# ---------------------------------------------------------------------------------


def int2ip(nn: int) -> str:
    """utils.Int2ip + net.IP.String(): LE u32 -> dotted quad (utils_linux.go:51-55)."""
    b = struct.pack("<I", nn & 0xFFFFFFFF)
    return "%d.%d.%d.%d" % (b[0], b[1], b[2], b[3])


def ip2int(s: str) -> int:
    """Inverse of int2ip (utils.Ip2int, utils_linux.go:57-62)."""
    a = [int(x) for x in s.split(".")]
    return a[0] | (a[1] << 8) | (a[2] << 16) | (a[3] << 24)


def host_to_net_short(i: int) -> int:
    """utils.HostToNetShort (utils_linux.go:65-70): byte swap of a u16."""
    return ((i & 0xFF) << 8) | ((i >> 8) & 0xFF)


def to_flow(src_ip: str, dst_ip: str, sport: int, dport: int, proto: int,
            obs: int, verdict: int) -> Flow:
    """utils.ToFlow (flow_utils.go:33-128)."""
    l4 = None
    if proto == 6:
        l4 = L4("TCP", sport, dport)
    elif proto == 17:
        l4 = L4("UDP", sport, dport)
    if obs == 0:
        point, direction = OBS_TO_STACK, TD_EGRESS
    elif obs == 1:
        point, direction = OBS_TO_ENDPOINT, TD_INGRESS
    elif obs == 2:
        point, direction = OBS_FROM_NETWORK, TD_INGRESS
    elif obs == 3:
        point, direction = OBS_TO_NETWORK, TD_EGRESS
    else:
        point, direction = OBS_UNKNOWN, TD_UNKNOWN
    if verdict == 0:
        verdict = VERDICT_FORWARDED
    return Flow(ip=IP(src_ip, dst_ip, 1), l4=l4, verdict=verdict, traffic_direction=direction,
                trace_observation_point=point, is_reply=False, extensions=RetinaMetadata())


def add_tcp_flags(f: Flow, syn, ack, fin, rst, psh, urg) -> None:
    """utils.AddTCPFlags (flow_utils.go:136-149): only for TCP L4; ECE/CWR never set."""
    if f.l4 is None or f.l4.proto != "TCP":
        return
    f.l4.flags = TCPFlags(FIN=fin == 1, SYN=syn == 1, RST=rst == 1, PSH=psh == 1,
                          ACK=ack == 1, URG=urg == 1)


# kernel TCP flag bits, pkg/plugin/packetparser/types_linux.go:22-31
TCP_FLAG_FIN, TCP_FLAG_SYN, TCP_FLAG_RST, TCP_FLAG_PSH, TCP_FLAG_ACK, TCP_FLAG_URG = (
    1, 2, 4, 8, 16, 32)

# struct packet, pkg/plugin/conntrack/_cprog/conntrack.c:34-49 (Go mirror
# packetparser_bpfel_x86.go:45-69): 72 bytes little-endian.
PACKET_STRUCT = struct.Struct("<QIIIHHIIIIBBBB?3xQQII")
assert PACKET_STRUCT.size == 72


def decode_packet(raw: bytes) -> Flow:
    """packetParser.processRecord decode (packetparser_linux.go:571-631)."""
    (t_nsec, nbytes, src, dst, sport, dport, seq, ack, tsval, tsecr, obs, tdir, proto,
     flags, is_reply, _bf, _br, _pf, _pr) = PACKET_STRUCT.unpack(raw)
    f = to_flow(int2ip(src), int2ip(dst), host_to_net_short(sport), host_to_net_short(dport),
                proto, obs, VERDICT_FORWARDED)
    f.is_reply = bool(is_reply)
    f.traffic_direction = tdir
    meta = RetinaMetadata(bytes=nbytes)
    add_tcp_flags(f, (flags & TCP_FLAG_SYN) >> 1, (flags & TCP_FLAG_ACK) >> 4,
                  flags & TCP_FLAG_FIN, (flags & TCP_FLAG_RST) >> 2,
                  (flags & TCP_FLAG_PSH) >> 3, (flags & TCP_FLAG_URG) >> 5)
    f.time_ns = t_nsec
    if f.trace_observation_point == OBS_TO_NETWORK:
        meta.tcp_id = tsval
    elif f.trace_observation_point == OBS_FROM_NETWORK:
        meta.tcp_id = tsecr
    f.extensions = meta
    return f


# struct packet of dropreason (drop_reason.c:39-54, Go kprobePacket): 32 bytes
# little-endian: src_ip, dst_ip, src_port, dst_port, skb_len, return_val, drop_type,
# proto, in_filtermap, ts.
DROP_STRUCT = struct.Struct("<IIHHIIHBBQ")
assert DROP_STRUCT.size == 32


def decode_drop(raw: bytes) -> Flow:
    """dropReason.processRecord decode (dropreason_linux.go:345-386): HostToNetShort on
    both ports, ToFlow(..., obs 2, DROPPED), AddDropReason(drop_type), AddPacketSize(skb_len)."""
    src, dst, sport, dport, skb_len, _ret, drop_type, proto, _infm, ts = DROP_STRUCT.unpack(raw)
    f = drop_flow(int2ip(src), int2ip(dst), host_to_net_short(sport), host_to_net_short(dport),
                  proto, drop_type, skb_len)
    f.time_ns = ts  # ToFlow(MonotonicOffset + Ts) (dropreason_linux.go:358-360), offset 0 here
    return f


# dropReason.processRecord after the decode: obs forced to 2, DROPPED.
def drop_flow(src_ip: str, dst_ip: str, sport: int, dport: int, proto: int,
              drop_type: int, skb_len: int) -> Flow:
    f = to_flow(src_ip, dst_ip, sport, dport, proto, 2, VERDICT_DROPPED)
    f.is_reply = None
    meta = RetinaMetadata(drop_reason=drop_type, bytes=skb_len)
    f.verdict = VERDICT_DROPPED  # AddDropReason (flow_utils.go:277-296)
    f.extensions = meta
    return f


def add_dns_info(f: Flow, meta: RetinaMetadata, qtype: str, rcode: int, query: str,
                 qtypes: List[str], num_answers: int, ips: List[str]) -> None:
    """utils.AddDNSInfo (flow_utils.go:186-220)."""
    f.dns = DNS(rcode=rcode, query=query, qtypes=list(qtypes), ips=list(ips))
    if qtype == "Q":
        meta.dns_type = DNS_TYPE_QUERY
        f.l7_type = "REQUEST"
    elif qtype == "R":
        meta.dns_type = DNS_TYPE_RESPONSE
        f.l7_type = "RESPONSE"
        f.is_reply = True
    else:
        meta.dns_type = DNS_TYPE_UNKNOWN
        f.l7_type = "UNKNOWN_L7_TYPE"
    meta.num_responses = num_answers
    f.extensions = meta


def get_dns(f: Optional[Flow]):
    """utils.GetDNS (flow_utils.go:222-234)."""
    if f is None or f.dns is None:
        return None, DNS_TYPE_UNKNOWN, 0
    if f.extensions is None:
        return f.dns, DNS_TYPE_UNKNOWN, 0
    return f.dns, f.extensions.dns_type, f.extensions.num_responses


DNS_RCODE_NAMES = {0: "NOERROR", 1: "FORMERR", 2: "SERVFAIL", 3: "NXDOMAIN", 4: "NOTIMP",
                   5: "REFUSED"}


def dns_rcode_to_string(f: Optional[Flow]) -> str:
    """utils.DNSRcodeToString (flow_utils.go:237-257)."""
    if f is None or f.dns is None:
        return ""
    return DNS_RCODE_NAMES.get(f.dns.rcode, "")


def packet_size(f: Flow) -> int:
    """utils.PacketSize (flow_utils.go:267-274)."""
    return 0 if f.extensions is None else f.extensions.bytes


def drop_reason_description(f: Optional[Flow]) -> str:
    """utils.DropReasonDescription (flow_utils.go:298-305)."""
    if f is None:
        return ""
    r = 0 if f.extensions is None else f.extensions.drop_reason
    return enum_string(DROP_REASON_NAMES, r)


# ---------------------------------------------------------------------------------
# a3 / a4: IP cache and enricher
# ---------------------------------------------------------------------------------


@dataclass
class RetinaEndpoint:
    """common.RetinaEndpoint subset (pkg/common/types.go:29-43, endpoint.go)."""
    name: str
    namespace: str
    ipv4: Optional[str] = None
    other_ipv4s: List[str] = field(default_factory=list)
    owner_refs: Optional[List[Workload]] = None
    labels: Dict[str, str] = field(default_factory=dict)

    def key(self) -> str:
        return self.namespace + "/" + self.name

    def ips(self) -> List[str]:
        """IPAddresses.GetIPs (ipaddr.go:35-50), IPv4 subset."""
        out = []
        if self.ipv4 is not None:
            out.append(self.ipv4)
        out.extend(self.other_ipv4s)
        return out


@dataclass
class RetinaSvc:
    name: str
    namespace: str
    ip: str

    def key(self) -> str:
        return self.namespace + "/" + self.name


@dataclass
class RetinaNode:
    name: str
    ip: str


class Cache:
    """controllers/cache.Cache IP maps (cache.go:17-46,110-169,204-420)."""

    def __init__(self):
        self.ip_to_ep_key: Dict[str, str] = {}
        self.ep_map: Dict[str, RetinaEndpoint] = {}
        self.ip_to_svc_key: Dict[str, str] = {}
        self.svc_map: Dict[str, RetinaSvc] = {}
        self.ip_to_node_name: Dict[str, str] = {}
        self.node_map: Dict[str, RetinaNode] = {}

    # -- lookups (cache.go:110-169)
    def get_obj_by_ip(self, ip: str):
        k = self.ip_to_ep_key.get(ip)
        if k is not None and k in self.ep_map:
            return self.ep_map[k]
        k = self.ip_to_svc_key.get(ip)
        if k is not None and k in self.svc_map:
            return self.svc_map[k]
        k = self.ip_to_node_name.get(ip)
        if k is not None and k in self.node_map:
            return self.node_map[k]
        return None

    # -- updates (cache.go:204-300)
    def update_retina_endpoint(self, ep: RetinaEndpoint) -> None:
        ips = ep.ips()
        if not ips:
            raise ValueError("no IP found for endpoint " + ep.key())
        for ip in ips:
            self._delete_by_ip(ip, ep.key())
        self.ep_map[ep.key()] = ep
        for ip in ips:
            self.ip_to_ep_key[ip] = ep.key()

    def update_retina_svc(self, svc: RetinaSvc) -> None:
        if not svc.ip:  # svc.GetPrimaryIP() error (cache.go:244-251)
            raise ValueError("no primary IP for service " + svc.key())
        self._delete_by_ip(svc.ip, svc.key())
        self.ip_to_svc_key[svc.ip] = svc.key()
        self.svc_map[svc.key()] = svc

    def update_retina_node(self, node: RetinaNode) -> None:
        self._delete_by_ip(node.ip, node.name)
        self.node_map[node.name] = node
        self.ip_to_node_name[node.ip] = node.name

    def delete_retina_endpoint(self, key: str) -> None:
        ep = self.ep_map.get(key)
        if ep is None:
            return
        del self.ep_map[key]
        for ip in ep.ips():
            self.ip_to_ep_key.pop(ip, None)

    def delete_retina_svc(self, key: str) -> None:  # deleteSvc (cache.go:347-371)
        if key not in self.svc_map:
            raise KeyError("service not found in cache: " + key)
        svc = self.svc_map.pop(key)
        self.ip_to_svc_key.pop(svc.ip, None)

    def delete_retina_node(self, name: str) -> None:  # deleteNode (cache.go:381-397)
        if name not in self.node_map:
            raise KeyError("node not found in cache: " + name)
        node = self.node_map.pop(name)
        self.ip_to_node_name.pop(node.ip, None)

    def _delete_by_ip(self, ip: str, key: str) -> None:
        """cache.deleteByIP (cache.go:395-420)."""
        if ip in self.ip_to_svc_key:
            if self.ip_to_svc_key[ip] == key:
                return
            self.delete_retina_svc(self.ip_to_svc_key[ip])
            return
        if ip in self.ip_to_ep_key:
            if self.ip_to_ep_key[ip] == key:
                return
            self.delete_retina_endpoint(self.ip_to_ep_key[ip])
            return
        if ip in self.ip_to_node_name:
            if self.ip_to_node_name[ip] == key:
                return
            self.delete_retina_node(self.ip_to_node_name[ip])


def get_endpoint(obj) -> Optional[Endpoint]:
    """Enricher.getEndpoint / getWorkloads (enricher.go:142-183)."""
    if isinstance(obj, RetinaEndpoint):
        wl = None
        if obj.owner_refs is not None:
            wl = [Workload(o.kind, o.name) for o in obj.owner_refs]
        return Endpoint(namespace=obj.namespace, pod_name=obj.name,
                        labels=["%s=%s" % kv for kv in obj.labels.items()], workloads=wl)
    return None


def enrich(cache: Cache, f: Flow) -> Optional[Flow]:
    """Enricher.enrich (enricher.go:102-135). Returns the exported flow, or None if dropped."""
    if f.ip.ip_version > 1:
        return None
    if f.ip.source == "":
        return None
    src = cache.get_obj_by_ip(f.ip.source)
    if src is not None:
        f.source = get_endpoint(src)
    if f.ip.destination == "":
        return None
    dst = cache.get_obj_by_ip(f.ip.destination)
    if dst is not None:
        f.destination = get_endpoint(dst)
    return f


# ---------------------------------------------------------------------------------
# a6: context options
# ---------------------------------------------------------------------------------

CTX_SOURCE, CTX_DESTINATION, CTX_LOCAL = 1, 2, 3
LOCAL_CONTEXT, REMOTE_CONTEXT = "local", "remote"
INGRESS, EGRESS = "ingress", "egress"


class ContextOptions:
    """ContextOptions (types.go:109-314)."""

    def __init__(self, opts: Optional[List[str]], option: int):
        self.option = option
        self.IP = self.Namespace = self.Podname = self.Workload = False
        self.Service = self.Port = False
        for o in opts or []:
            o = o.lower()
            if o == "ip":
                self.IP = True
            elif o == "namespace":
                self.Namespace = True
            elif o == "podname":
                self.Podname = True
            elif o == "workload":
                self.Workload = True
            elif o == "service":
                self.Service = True
            elif o == "port":
                self.Port = True

    def get_labels(self) -> List[str]:
        prefix = {CTX_SOURCE: "source_", CTX_DESTINATION: "destination_"}.get(self.option, "")
        labels = []
        if self.IP:
            labels.append(prefix + "ip")
        if self.Namespace:
            labels.append(prefix + "namespace")
        if self.Podname:
            labels.append(prefix + "podname")
        if self.Workload:
            labels += [prefix + "workload_kind", prefix + "workload_name"]
        if self.Service:
            labels.append(prefix + "service")
        if self.Port:
            labels.append(prefix + "port")
        return labels

    def get_values(self, f: Optional[Flow]) -> List[str]:
        return self.get_by_direction_values(f, self.option == CTX_DESTINATION)

    def get_local_ctx_values(self, f: Optional[Flow]) -> Optional[Dict[str, Optional[List[str]]]]:
        values = {INGRESS: None, EGRESS: None}
        if self.option != CTX_LOCAL:
            return None
        if f is None:
            return values
        if f.source is not None and not is_apiserver_pod(f.source):
            values[EGRESS] = self.get_by_direction_values(f, False)
        if f.destination is not None and not is_apiserver_pod(f.destination):
            values[INGRESS] = self.get_by_direction_values(f, True)
        return values

    def get_by_direction_values(self, f: Optional[Flow], dest: bool) -> List[str]:
        values: List[str] = []
        if f is None:
            return values
        if self.IP:
            ip = "unknown"
            if f.ip is not None:
                ip = f.ip.destination if dest else f.ip.source
            values.append(ip)
        ep = f.destination if dest else f.source
        if self.Namespace:
            values.append(ep.namespace if ep is not None else "unknown")
        if self.Podname:
            values.append(ep.pod_name if ep is not None else "unknown")
        if self.Workload:
            wk = ep.workloads if ep is not None else None
            if wk:
                values += [wk[0].kind, wk[0].name]
            else:
                values += ["unknown", "unknown"]
        if self.Service:
            values.append("unknown")  # flow.{Source,Destination}Service is never set
        if self.Port:
            if f.l4 is not None:
                values.append(str(f.l4.destination_port if dest else f.l4.source_port))
            else:
                values.append("unknown")
        return values


def is_apiserver_pod(ep: Optional[Endpoint]) -> bool:
    """types.go:358-368."""
    return (ep is not None and ep.namespace == APISERVER_ENDPOINT_NAME
            and ep.pod_name == APISERVER_ENDPOINT_NAME)


# ---------------------------------------------------------------------------------
# a7-a12: metrics
# ---------------------------------------------------------------------------------


class Vec:
    """Prometheus GaugeVec / CounterVec: label tuple -> accumulated value (exact int)."""

    def __init__(self, name: str, label_names: List[str]):
        self.name = RETINA_NAMESPACE + "_" + name
        self.label_names = list(label_names)
        self.series: Dict[Tuple[str, ...], int] = {}
        self.calls = 0

    def add(self, values: List[str], v: int) -> None:
        if len(values) != len(self.label_names):
            raise ValueError("inconsistent label cardinality for %s: %r vs %r"
                             % (self.name, values, self.label_names))
        t = tuple(values)
        self.series[t] = self.series.get(t, 0) + v
        self.calls += 1


@dataclass
class MetricsContextOptions:
    """crd/api/v1alpha1 MetricsContextOptions (metricsconfiguration_types.go:27-58)."""
    metric_name: str = ""
    source_labels: Optional[List[str]] = None
    destination_labels: Optional[List[str]] = None

    def is_advanced(self) -> bool:  # metricsconfiguration_types.go:97-101
        return self.metric_name != "" and (len(self.source_labels or []) > 0
                                           or len(self.destination_labels or []) > 0)


class BaseMetric:
    """baseMetricObject (basemetricsobject.go:19-53)."""

    def __init__(self, opts: MetricsContextOptions, ctx: str):
        self.adv_enable = opts.is_advanced()
        self.context_mode = ctx
        self.src_ctx = self.dst_ctx = None
        if ctx == LOCAL_CONTEXT:
            if opts.source_labels is not None:
                self.src_ctx = ContextOptions(opts.source_labels, CTX_LOCAL)
        else:
            if opts.source_labels is not None:
                self.src_ctx = ContextOptions(opts.source_labels, CTX_SOURCE)
            if opts.destination_labels is not None:
                self.dst_ctx = ContextOptions(opts.destination_labels, CTX_DESTINATION)
        self.metric_name = ""
        self.vec: Optional[Vec] = None

    def is_local(self) -> bool:
        return self.context_mode == LOCAL_CONTEXT

    def _ctx_labels(self) -> List[str]:
        out = []
        if self.src_ctx is not None:
            out += self.src_ctx.get_labels()
        if self.dst_ctx is not None:
            out += self.dst_ctx.get_labels()
        return out

    def _ctx_values(self, f: Flow) -> List[str]:
        out = []
        if self.src_ctx is not None:
            out += self.src_ctx.get_values(f)
        if self.dst_ctx is not None:
            out += self.dst_ctx.get_values(f)
        return out


class ForwardMetrics(BaseMetric):
    """forward.go:88-224."""

    @staticmethod
    def new(opts, ctx):
        if opts is None or "forward" not in opts.metric_name.lower():
            return None
        return ForwardMetrics(opts, ctx)

    def init(self, metric_name: str) -> None:
        if metric_name == FORWARD_PACKETS_GAUGE:
            self.vec = Vec("adv_forward_count", self.get_labels())
        elif metric_name == FORWARD_BYTES_GAUGE:
            self.vec = Vec("adv_forward_bytes", self.get_labels())
        self.metric_name = metric_name

    def get_labels(self) -> List[str]:
        labels = ["direction"]
        if not self.adv_enable:
            return labels
        return labels + self._ctx_labels()

    def process_flow(self, f: Optional[Flow]) -> None:
        if f is None or f.verdict != VERDICT_FORWARDED:
            return
        if self.is_local():
            m = self.src_ctx.get_local_ctx_values(f)
            if m is None:
                return
            if m[INGRESS]:
                self._update(f, [INGRESS] + m[INGRESS])
            if m[EGRESS]:
                self._update(f, [EGRESS] + m[EGRESS])
            return
        labels = [traffic_direction_string(f.traffic_direction)]
        if self.adv_enable:
            labels += self._ctx_values(f)
        self._update(f, labels)

    def _update(self, f: Flow, labels: List[str]) -> None:
        if self.metric_name == FORWARD_PACKETS_GAUGE:
            self.vec.add(labels, 1)
        elif self.metric_name == FORWARD_BYTES_GAUGE:
            self.vec.add(labels, packet_size(f))


class DropCountMetrics(BaseMetric):
    """drops.go:91-171."""

    @staticmethod
    def new(opts, ctx):
        if opts is None or "drop" not in opts.metric_name.lower():
            return None
        return DropCountMetrics(opts, ctx)

    def init(self, metric_name: str) -> None:
        if metric_name == DROPPED_PACKETS_GAUGE:
            self.vec = Vec("adv_drop_count", self.get_labels())
        elif metric_name == DROP_BYTES_GAUGE:
            self.vec = Vec("adv_drop_bytes", self.get_labels())
        self.metric_name = metric_name

    def get_labels(self) -> List[str]:
        return ["reason", "direction"] + self._ctx_labels()

    def process_flow(self, f: Optional[Flow]) -> None:
        if f is None or f.verdict != VERDICT_DROPPED:
            return
        if self.is_local():
            m = self.src_ctx.get_local_ctx_values(f)
            if m is None:
                return
            reason = drop_reason_description(f)
            if m[INGRESS]:
                self._update(f, [reason, INGRESS] + m[INGRESS])
            if m[EGRESS]:
                self._update(f, [reason, EGRESS] + m[EGRESS])
            return
        labels = [drop_reason_description(f), traffic_direction_string(f.traffic_direction)]
        if self.adv_enable:
            labels += self._ctx_values(f)
        self._update(f, labels)

    def _update(self, f: Flow, labels: List[str]) -> None:
        if self.metric_name == DROPPED_PACKETS_GAUGE:
            self.vec.add(labels, 1)
        elif self.metric_name == DROP_BYTES_GAUGE:
            self.vec.add(labels, packet_size(f))


def tcp_flag_values(flags: Optional[TCPFlags]) -> List[str]:
    """TCPMetrics.getFlagValues (tcpflags.go:134-175)."""
    out: List[str] = []
    if flags is None:
        return out
    if flags.FIN:
        out.append(FLAG_FIN)
    if flags.SYN and flags.ACK:
        out.append(FLAG_SYNACK)
    else:
        if flags.SYN:
            out.append(FLAG_SYN)
        if flags.ACK:
            out.append(FLAG_ACK)
    if flags.RST:
        out.append(FLAG_RST)
    if flags.PSH:
        out.append(FLAG_PSH)
    if flags.URG:
        out.append(FLAG_URG)
    if flags.ECE:
        out.append(FLAG_ECE)
    if flags.CWR:
        out.append(FLAG_CWR)
    return out


class TCPMetrics(BaseMetric):
    """tcpflags.go:31-179."""

    @staticmethod
    def new(opts, ctx):
        if opts is None or "flag" not in opts.metric_name.lower():
            return None
        return TCPMetrics(opts, ctx)

    def init(self, metric_name: str) -> None:
        self.vec = Vec("adv_tcpflags_count", self.get_labels())

    def get_labels(self) -> List[str]:
        return ["flag"] + self._ctx_labels()

    def process_flow(self, f: Optional[Flow]) -> None:
        if f is None or f.verdict != VERDICT_FORWARDED:
            return
        if f.l4 is None or f.l4.proto != "TCP":
            return
        flags = tcp_flag_values(f.l4.flags)
        if not flags:
            return
        if self.is_local():
            m = self.src_ctx.get_local_ctx_values(f)
            if m is None:
                return
            if m[INGRESS]:
                for fl in flags:
                    self.vec.add([fl] + m[INGRESS], 1)
            if m[EGRESS]:
                for fl in flags:
                    self.vec.add([fl] + m[EGRESS], 1)
            return
        src = self.src_ctx.get_values(f) if self.src_ctx is not None else []
        dst = self.dst_ctx.get_values(f) if self.dst_ctx is not None else []
        for fl in flags:
            self.vec.add([fl] + src + dst, 1)


class TCPRetransMetrics(BaseMetric):
    """tcpretrans.go:68-119."""

    @staticmethod
    def new(opts, ctx):
        if opts is None or "retrans" not in opts.metric_name.lower():
            return None
        return TCPRetransMetrics(opts, ctx)

    def init(self, metric_name: str) -> None:
        self.vec = Vec("adv_tcpretrans_count", self.get_labels())

    def get_labels(self) -> List[str]:
        return ["direction"] + self._ctx_labels()

    def process_flow(self, f: Optional[Flow]) -> None:
        if f is None or f.verdict != VERDICT_RETRANSMISSION:
            return
        if self.is_local():
            m = self.src_ctx.get_local_ctx_values(f)
            if m is None:
                return
            if m[INGRESS]:
                self.vec.add([INGRESS] + m[INGRESS], 1)
            if m[EGRESS]:
                self.vec.add([EGRESS] + m[EGRESS], 1)
            return
        self.vec.add([traffic_direction_string(f.traffic_direction)] + self._ctx_values(f), 1)


class DNSMetrics(BaseMetric):
    """dns.go:102-238."""

    @staticmethod
    def new(opts, ctx):
        if opts is None or "dns" not in opts.metric_name.lower():
            return None
        return DNSMetrics(opts, ctx)

    def init(self, metric_name: str) -> None:
        self.metric_name = metric_name
        if metric_name == DNS_REQUEST_COUNTER:
            self.vec = Vec("adv_" + DNS_REQUEST_COUNTER, DNS_REQUEST_LABELS + self._ctx_labels())
        elif metric_name == DNS_RESPONSE_COUNTER:
            self.vec = Vec("adv_" + DNS_RESPONSE_COUNTER, DNS_RESPONSE_LABELS + self._ctx_labels())

    def _type_ok(self, dns_type: int) -> bool:
        if dns_type == DNS_TYPE_UNKNOWN:
            return False
        if self.metric_name == DNS_REQUEST_COUNTER and dns_type != DNS_TYPE_QUERY:
            return False
        if self.metric_name == DNS_RESPONSE_COUNTER and dns_type != DNS_TYPE_RESPONSE:
            return False
        return True

    def request_values(self, f: Optional[Flow]) -> Optional[List[str]]:
        dns, t, _ = get_dns(f)
        if dns is None or not self._type_ok(t):
            return None
        return [",".join(dns.qtypes), dns.query]

    def response_values(self, f: Optional[Flow]) -> Optional[List[str]]:
        dns, t, n = get_dns(f)
        if dns is None or not self._type_ok(t):
            return None
        return [dns_rcode_to_string(f), ",".join(dns.qtypes), dns.query, ",".join(dns.ips), str(n)]

    def _labels_for_flow(self, f: Flow) -> Optional[List[str]]:
        t = f.extensions.dns_type if f.extensions is not None else DNS_TYPE_UNKNOWN
        if t == DNS_TYPE_QUERY:
            return self.request_values(f)
        if t == DNS_TYPE_RESPONSE:
            return self.response_values(f)
        return None

    def process_flow(self, f: Optional[Flow]) -> None:
        if f is None or f.verdict != VERDICT_DNS:
            return
        if self.is_local():
            self.process_local_ctx_flow(f)
            return
        labels = self._labels_for_flow(f)
        if not labels:
            return
        self.vec.add(labels + self._ctx_values(f), 1)

    def process_local_ctx_flow(self, f: Flow) -> None:
        m = self.src_ctx.get_local_ctx_values(f)
        if m is None:
            return
        labels = self._labels_for_flow(f)
        if not labels:
            return
        if m[INGRESS] and m[EGRESS]:
            if f.traffic_direction == TD_INGRESS:
                labels = labels + m[INGRESS]
            else:
                labels = labels + m[EGRESS]
        elif m[INGRESS]:
            labels = labels + m[INGRESS]
        elif m[EGRESS]:
            labels = labels + m[EGRESS]
        else:
            return
        self.vec.add(labels, 1)


def _same_set(a: Optional[List[str]], b: Optional[List[str]]) -> bool:
    """utils.CompareStringSlice (pkg/utils/common.go:58-84): equal lengths and equal sets."""
    a, b = list(a or []), list(b or [])
    return len(a) == len(b) and set(a) == set(b)


def options_equal(old: List[MetricsContextOptions], new: List[MetricsContextOptions]) -> bool:
    """validations.MetricsContextOptionsCompare (validate_metricconfiguration.go:118-162)."""
    if len(old) != len(new):
        return False
    om = {o.metric_name: o for o in old}
    nm = {o.metric_name: o for o in new}
    if len(om) != len(nm):
        return False
    for k, o in om.items():
        n = nm.get(k)
        if n is None or not _same_set(o.source_labels, n.source_labels) \
                or not _same_set(o.destination_labels, n.destination_labels):
            return False
    return True


class Module:
    """metrics.Module registry + per-flow dispatch (metrics_module.go:205-305)."""

    def __init__(self, remote_context: bool = False):
        self.ctx = REMOTE_CONTEXT if remote_context else LOCAL_CONTEXT
        self.registry: Dict[str, BaseMetric] = {}
        self.current_spec: Optional[List[MetricsContextOptions]] = None

    def reconcile_spec(self, context_options: List[MetricsContextOptions]) -> bool:
        """Module.Reconcile (metrics_module.go:142-170): nothing happens when the spec equals
        currentSpec, or -- with a currentSpec -- when MetricsContextOptionsCompare finds the
        options equal (validate_metricconfiguration.go:118-162: same metric names, label
        lists equal as sets); otherwise updateMetricsContexts rebuilds the registry.
        Returns whether the registry was rebuilt."""
        rebuild = self.current_spec is None or not options_equal(self.current_spec, context_options)
        if rebuild:
            self.reconcile(context_options)
        self.current_spec = list(context_options)
        return rebuild

    def reconcile(self, context_options: List[MetricsContextOptions]) -> None:
        self.registry = {}
        for o in context_options:
            name = o.metric_name
            if "forward" in name:
                m = ForwardMetrics.new(o, self.ctx)
                if m is not None:
                    self.registry[name] = m
            elif "drop" in name:
                m = DropCountMetrics.new(o, self.ctx)
                if m is not None:
                    self.registry[name] = m
            elif "tcp" in name:
                m = TCPMetrics.new(o, self.ctx)
                if m is not None:
                    self.registry[name] = m
                m = TCPRetransMetrics.new(o, self.ctx)
                if m is not None:
                    self.registry[name] = m
            elif "node_apiserver" in name:
                pass  # latency metrics: out of scope
            elif "dns" in name or "pktmon" in name:
                m = DNSMetrics.new(o, self.ctx)
                if m is not None:
                    self.registry[name] = m
        for name, m in self.registry.items():
            m.init(name)

    def process_flow(self, f: Flow) -> None:
        for m in self.registry.values():
            m.process_flow(f)

    def series(self) -> Dict[Tuple[str, Tuple[Tuple[str, str], ...]], int]:
        """Every (metric, ((label, value), ...)) series with its exact integer value."""
        out = {}
        for m in self.registry.values():
            if m.vec is None:
                continue
            for vals, v in m.vec.series.items():
                out[(m.vec.name, tuple(zip(m.vec.label_names, vals)))] = v
        return out
