"""Hubble-mode L3/L4 enrichment, restated (TEST INFRASTRUCTURE ONLY).

Follows pkg/hubble/parser/layer34/parser_linux.go and pkg/hubble/common/decoder_linux.go:
  * Parser.Decode (:30-57): flows without IP are returned unchanged; otherwise Source and
    Destination are replaced by epDecoder.Decode of each address, then decodeSummary;
  * epDecoder.Decode (decoder_linux.go:32-60): PodName / Namespace from the ipcache's K8s
    metadata when present; identity = ipcache.LookupByIP, World when absent; ID and
    Identity both set to it; Labels: the reserved label set for host / kube-apiserver /
    remote-node / world, else the ipcache's metadata labels of the IP;
  * decodeSummary (:59-84): DROPPED flows get EventType.SubType = DropReasonDesc and
    Summary "Drop Reason: <desc>\\nNote: ..." (only when EventType is set, which ToFlow
    always does); TCP flows with flags get "TCP Flags: " + TCPFlags.String(); UDP flows
    get "UDP".

Constants from cilium (pinned in go.mod, absent from this image): reserved identities
host 1, world 2, remote-node 6, kube-apiserver 7 and their label sets "reserved:host",
"reserved:world", "reserved:remote-node", "reserved:kube-apiserver".  TCPFlags.String() is
the protobuf text form of the set fields ("SYN:true ACK:true").  These three are *parity
unpinned*: the reference has no test for this parser and cilium is not importable here.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from . import oracle as O

ID_HOST, ID_WORLD, ID_REMOTE_NODE, ID_KUBE_APISERVER = 1, 2, 6, 7
RESERVED_LABELS = {ID_HOST: ["reserved:host"], ID_WORLD: ["reserved:world"],
                   ID_REMOTE_NODE: ["reserved:remote-node"], ID_KUBE_APISERVER: ["reserved:kube-apiserver"]}
DROP_NOTE = "\nNote: This reason is most accurate. Prefer over others while using Hubble CLI."
# summary codes of the engine (include/gpuagg.h gpuagg_hubble_cols.summary_kind)
SUM_NONE, SUM_TCP, SUM_UDP, SUM_DROP, SUM_DNS = 0, 1, 2, 3, 4
# gopacket layers.DNSResponseCode.String() (*parity unpinned*: gopacket is not in the image)
DNS_RCODE_NAMES = {0: "No Error", 1: "Format Error", 2: "Server Failure", 3: "Non-Existent Domain",
                   4: "Not Implemented", 5: "Query Refused"}


@dataclass
class IPCacheEntry:
    identity: int
    meta: Optional[int] = None             # K8s metadata id (pod, namespace) or None
    labels: List[str] = field(default_factory=list)


@dataclass
class HubbleEndpoint:
    id: int
    identity: int
    pod_name: str = ""
    namespace: str = ""
    labels: List[str] = field(default_factory=list)


def decode_endpoint(ipcache: Dict[str, IPCacheEntry], meta: Dict[int, Tuple[str, str]], ip: str) -> HubbleEndpoint:
    """epDecoder.Decode (decoder_linux.go:32-60)."""
    e = ipcache.get(ip)
    ep = HubbleEndpoint(0, 0)
    if e is not None and e.meta is not None:
        ep.pod_name, ep.namespace = meta[e.meta]
    ident = e.identity if e is not None else ID_WORLD
    ep.id = ep.identity = ident
    ep.labels = list(RESERVED_LABELS[ident]) if ident in RESERVED_LABELS else list(e.labels if e else [])
    return ep


def tcp_flags_string(f: O.TCPFlags) -> str:
    """protobuf text of flow.TCPFlags: set fields in declaration order (FIN SYN RST PSH
    ACK URG ECE CWR NS)."""
    parts = [n for n, v in (("FIN", f.FIN), ("SYN", f.SYN), ("RST", f.RST), ("PSH", f.PSH),
                            ("ACK", f.ACK), ("URG", f.URG)) if v]
    return " ".join("%s:true" % n for n in parts)


def dns_summary(dns: O.DNS, l7_type: str) -> str:
    """seven.dnsSummary (seven/parser_linux.go:117-146)."""
    if not dns.qtypes:
        return ""
    q = ",".join(dns.qtypes)
    if l7_type == "REQUEST":
        return "DNS Query %s %s" % (dns.query, q)
    if l7_type == "RESPONSE":
        if dns.rcode != 0:
            answer = "RCode: %s" % DNS_RCODE_NAMES.get(dns.rcode, "Unknown")
        else:
            parts = []
            if dns.ips:
                parts.append('"%s"' % ",".join(dns.ips))  # %q of a plain ASCII string
            answer = " ".join(parts)
        return "DNS Answer %s (Query %s %s)" % (answer, dns.query, q)
    return ""


def summary(f: O.Flow) -> Tuple[int, int, str]:
    """Parser._decode (parser_linux.go:64-93): L7 flows (DNS) through seven.Parser
    (dnsSummary), L3/L4 flows through decodeSummary (:59-84) -> (engine code, payload,
    summary string)."""
    if f.dns is not None:
        return SUM_DNS, 0, dns_summary(f.dns, f.l7_type)
    if f.verdict == O.VERDICT_DROPPED:
        r = f.extensions.drop_reason if f.extensions is not None else 0
        return SUM_DROP, r, "Drop Reason: %s%s" % (O.drop_reason_description(f), DROP_NOTE)
    if f.l4 is not None:
        if f.l4.proto == "TCP":
            if f.l4.flags is not None:
                fl = f.l4.flags
                mask = (fl.FIN << 0) | (fl.SYN << 1) | (fl.RST << 2) | (fl.PSH << 3) | (fl.ACK << 4) | (fl.URG << 5)
                return SUM_TCP, int(mask), "TCP Flags: " + tcp_flags_string(fl)
            return SUM_NONE, 0, ""
        if f.l4.proto == "UDP":
            return SUM_UDP, 0, "UDP"
    return SUM_NONE, 0, ""


def render_summary(code: int, payload: int) -> str:
    """The summary string of an engine summary word (host side of the Go binding)."""
    if code == SUM_DROP:
        return "Drop Reason: %s%s" % (O.enum_string(O.DROP_REASON_NAMES, payload), DROP_NOTE)
    if code == SUM_TCP:
        fl = O.TCPFlags(FIN=bool(payload & 1), SYN=bool(payload & 2), RST=bool(payload & 4),
                        PSH=bool(payload & 8), ACK=bool(payload & 16), URG=bool(payload & 32))
        return "TCP Flags: " + tcp_flags_string(fl)
    if code == SUM_UDP:
        return "UDP"
    return ""
