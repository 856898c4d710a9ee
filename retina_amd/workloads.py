"""Seeded synthetic flow batches for the BASELINE.json configs.

All inputs are numpy PCG64-seeded; nothing is downloaded.  Records follow the column
contract of include/gpuagg.h (src_ip/dst_ip as LE u32 of the network-order bytes).

* C1: 1M IPv4 TCP records, 10k pods, local ctx [ip, namespace, podname, workload]
* C2: 100M records, 10k pods, per-pod forward count/bytes + drop-reason histogram
* C3: records for count-min (d=4, w=2^20) + HLL p=14 distinct-dst per source pod
* C4: C2 shape with Zipf(1.2) source pods and 5-tuple ranks
* C5: 100k pods, 60% forwarded TCP, 5% retransmits, 35% DNS query/response
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .engine import Endpoint

PROTO_TCP, PROTO_UDP, PROTO_ICMP = 6, 17, 1
V_FWD, V_DROP, V_RETRANS, V_DNS = 1, 2, 15, 16
FIN, SYN, RST, PSH, ACK, URG = 1, 2, 4, 8, 16, 32
FLAG_COMBOS = np.array([SYN, SYN | ACK, ACK, ACK | PSH, FIN | ACK, RST], np.uint32)
APISERVER = "kubernetes-apiserver"


def ip_le(a: int, b: int, c: int, d: int) -> int:
    return a | (b << 8) | (c << 16) | (d << 24)


def pack_meta(proto, verdict, tdir=0, reason=0, flags=0, is_reply=0, dns_type=0, obs=0):
    """meta word of include/gpuagg.h (vectorised over numpy arrays)."""
    u = np.uint32
    return (np.asarray(proto, u) & u(0xFF)) | ((np.asarray(verdict, u) & u(0xFF)) << u(8)) \
        | ((np.asarray(tdir, u) & u(3)) << u(16)) | ((np.asarray(reason, u) & u(7)) << u(18)) \
        | ((np.asarray(flags, u) & u(0x3F)) << u(21)) | ((np.asarray(is_reply, u) & u(1)) << u(27)) \
        | ((np.asarray(dns_type, u) & u(3)) << u(28)) | ((np.asarray(obs, u) & u(3)) << u(30))


@dataclass
class Pods:
    endpoints: List[Endpoint]
    ips: np.ndarray          # every pod IP (primary + secondary), u32
    ip_owner: np.ndarray     # endpoint index per entry of ips


def make_pods(n_pods: int, seed: int = 0, secondary_frac: float = 0.05, owner_frac: float = 0.9,
              apiserver: bool = True, n_namespaces: int = 100) -> Pods:
    """Pod i: 10.(i>>16).(i>>8&255).(i&255); 5% also 10.(128+(i>>16)).(..) (ipaddr.go:35-50)."""
    rng = np.random.Generator(np.random.PCG64(seed + 1000))
    sec = rng.random(n_pods) < secondary_frac
    owned = rng.random(n_pods) < owner_frac
    eps: List[Endpoint] = []
    ips: List[int] = []
    owner_idx: List[int] = []
    for i in range(n_pods):
        prim = ip_le(10, (i >> 16) & 255, (i >> 8) & 255, i & 255)
        pip = [prim]
        if sec[i]:
            pip.append(ip_le(10, 128 + ((i >> 16) & 127), (i >> 8) & 255, i & 255))
        if apiserver and i == 0:
            ep = Endpoint(APISERVER, APISERVER, pip, None)
        else:
            ep = Endpoint("ns-%d" % (i % n_namespaces), "pod-%d" % i, pip,
                          [("ReplicaSet", "rs-%d" % (i // 10))] if owned[i] else None)
        eps.append(ep)
        ips.extend(pip)
        owner_idx.extend([i] * len(pip))
    return Pods(eps, np.array(ips, np.uint32), np.array(owner_idx, np.int64))


@dataclass
class DnsPayload:
    rcode: int
    qtypes: List[str]
    query: str
    ips: List[str]
    num_answers: int


@dataclass
class Records:
    src_ip: np.ndarray
    dst_ip: np.ndarray
    bytes: np.ndarray
    meta: np.ndarray
    ports: np.ndarray
    dns_id: np.ndarray
    dns: List[DnsPayload] = field(default_factory=list)
    tcp_id: Optional[np.ndarray] = None   # u32, latency metrics
    time_ns: Optional[np.ndarray] = None  # u64, latency metrics

    def __len__(self) -> int:
        return int(self.src_ip.shape[0])


def _pick_ips(rng, n: int, pods: Pods, pod_frac: float, zipf: Optional[float]) -> np.ndarray:
    is_pod = rng.random(n) < pod_frac
    if zipf:
        idx = (rng.zipf(zipf, n) - 1) % len(pods.ips)
    else:
        idx = rng.integers(0, len(pods.ips), n)
    ext = (np.uint32(100) | (rng.integers(64, 128, n, dtype=np.uint32) << np.uint32(8))
           | (rng.integers(0, 256, n, dtype=np.uint32) << np.uint32(16))
           | (rng.integers(1, 255, n, dtype=np.uint32) << np.uint32(24)))
    return np.where(is_pod, pods.ips[idx], ext).astype(np.uint32)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x += np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return x


def flow_tuples(flow_id: np.ndarray, pods: Pods, n_dst: int, udp_frac: float = 0.0):
    """The fixed 5-tuple of each flow id (C3, SURVEY.md 8d: flows with src in the pods and
    dst among n_dst IPs, the first len(pods.ips) of them the pod IPs): a pure function of
    the id, so a flow has the same 5-tuple in every chunk and on every rank."""
    u = np.uint32
    h1 = _splitmix64(flow_id)
    h2 = _splitmix64(flow_id ^ np.uint64(0x5851F42D4C957F2D))
    src = pods.ips[(h1 % np.uint64(len(pods.ips))).astype(np.int64)]
    j = (h2 % np.uint64(n_dst)).astype(np.int64)
    npi = len(pods.ips)
    k = np.maximum(j - npi, 0).astype(u)
    ext = (u(100) | ((u(64) + (k >> u(16))) << u(8)) | (((k >> u(8)) & u(255)) << u(16))
           | ((k & u(255)) << u(24)))
    dst = np.where(j < npi, pods.ips[np.minimum(j, npi - 1)], ext).astype(u)
    h3 = (h1 >> np.uint64(32)).astype(u)
    sport = u(32768) + (h3 % u(28232))
    dport = np.array([80, 443, 53, 8080, 6443, 9090], u)[((h2 >> np.uint64(40)) % np.uint64(6)).astype(np.int64)]
    udp = ((h2 >> np.uint64(8)) & np.uint64(0xFFFF)).astype(np.float64) < udp_frac * 65536.0
    return src, dst, (sport | (dport << u(16))).astype(u), udp


def gen_records(n: int, pods: Pods, seed: int, *, pod_frac: float = 0.8, drop_frac: float = 0.10,
                retrans_frac: float = 0.0, dns_frac: float = 0.0, udp_frac: float = 0.0,
                other_proto_frac: float = 0.0, zipf: Optional[float] = None,
                n_queries: int = 100_000, odd_frac: float = 0.0, flows: Optional[int] = None,
                n_dst: int = 1_000_000, flow_zipf: Optional[float] = None) -> Records:
    """Vectorised record generator (SURVEY.md 8d distributions).

    odd_frac adds edge rows: unknown / out-of-range traffic directions, verdicts no
    metric consumes, drop reason 7, destination 255.255.255.255.
    flows: draw each record's 5-tuple from `flows` fixed flows (flow_tuples; uniform, or
    Zipf(flow_zipf) over flow ranks) instead of independently per record."""
    rng = np.random.Generator(np.random.PCG64(seed))
    u = np.uint32
    if flows:
        fid = ((rng.zipf(flow_zipf, n) - 1) % flows) if flow_zipf else rng.integers(0, flows, n)
        src, dst, ports_f, udp_f = flow_tuples(fid.astype(np.uint64), pods, n_dst, udp_frac)
    else:
        src = _pick_ips(rng, n, pods, pod_frac, zipf)
        dst = _pick_ips(rng, n, pods, pod_frac, None)
    nbytes = rng.integers(64, 1501, n, dtype=u)
    r = rng.random(n)
    verdict = np.full(n, V_FWD, u)
    verdict[r < drop_frac] = V_DROP
    verdict[(r >= drop_frac) & (r < drop_frac + retrans_frac)] = V_RETRANS
    is_dns = (r >= drop_frac + retrans_frac) & (r < drop_frac + retrans_frac + dns_frac)
    verdict[is_dns] = V_DNS
    pr = rng.random(n)
    proto = np.full(n, PROTO_TCP, u)
    proto[pr < udp_frac] = PROTO_UDP
    proto[(pr >= udp_frac) & (pr < udp_frac + other_proto_frac)] = PROTO_ICMP
    if flows:  # the flow fixes its protocol
        proto = np.where(udp_f, u(PROTO_UDP), u(PROTO_TCP))
    proto[is_dns] = PROTO_UDP
    tdir = rng.integers(1, 3, n, dtype=u)
    tdir[verdict == V_DROP] = 1       # dropreason: obs 2 -> INGRESS (dropreason_linux.go:358-368)
    tdir[verdict == V_RETRANS] = 2    # tcpretrans: obs 0 -> EGRESS (tcpretrans_linux.go:124-134)
    reason = np.where(verdict == V_DROP, rng.integers(0, 7, n, dtype=u), u(0))
    flags = FLAG_COMBOS[rng.integers(0, len(FLAG_COMBOS), n)]
    flags = np.where((proto == PROTO_TCP) & ((verdict == V_FWD) | (verdict == V_RETRANS)), flags, u(0))
    is_reply = rng.integers(0, 2, n, dtype=u)
    sport = rng.integers(32768, 61000, n, dtype=u)
    dport = np.array([80, 443, 53, 8080, 6443, 9090], u)[rng.integers(0, 6, n)]
    dns_type = np.zeros(n, u)
    dns_id = np.zeros(n, u)
    payloads: List[DnsPayload] = []
    if is_dns.any():
        k = int(is_dns.sum())
        dns_type[is_dns] = rng.integers(1, 3, k, dtype=u)
        q = (rng.zipf(1.1, k) - 1) % n_queries
        qt = rng.integers(0, 3, k)
        rc = rng.integers(0, 6, k)
        na = rng.integers(0, 5, k)
        resp = dns_type[is_dns] == 2
        tdir[is_dns] = np.where(resp, u(1), u(2))  # responses HOST(obs 2), queries OUTGOING(obs 3)
        qtypes = ["A", "AAAA", "CNAME"]
        index: Dict[Tuple, int] = {}
        ids = np.empty(k, u)
        for j in range(k):
            if resp[j]:
                ipsl = ["10.%d.%d.%d" % (1 + (int(q[j]) >> 16), (int(q[j]) >> 8) & 255, (int(q[j]) + a) & 255)
                        for a in range(int(na[j]))]
                key = (int(rc[j]), int(qt[j]), int(q[j]), int(na[j]))
                p = (int(rc[j]), [qtypes[qt[j]]], "q%d.example.com" % q[j], ipsl, int(na[j]))
            else:  # same key as a rcode-0, no-answer response: identical label payload
                key = (0, int(qt[j]), int(q[j]), 0)
                p = (0, [qtypes[qt[j]]], "q%d.example.com" % q[j], [], 0)
            i = index.get(key)
            if i is None:
                i = len(payloads)
                index[key] = i
                payloads.append(DnsPayload(*p))
            ids[j] = i
        dns_id[is_dns] = ids
    if odd_frac:
        o = rng.random(n) < odd_frac
        kinds = rng.integers(0, 4, n)
        tdir = np.where(o & (kinds == 0), rng.integers(0, 4, n, dtype=u), tdir)
        verdict = np.where(o & (kinds == 1), np.array([0, 3, 4, 99], u)[rng.integers(0, 4, n)], verdict)
        reason = np.where(o & (kinds == 2) & (verdict == V_DROP), u(7), reason)
        dst = np.where(o & (kinds == 3), u(0xFFFFFFFF), dst)
    meta = pack_meta(proto, verdict, tdir, reason, flags, is_reply, dns_type)
    ports = ports_f if flows else (sport | (dport << u(16))).astype(u)
    return Records(src, dst, nbytes, meta.astype(u), ports, dns_id, payloads)


# ---- raw perf records (GPUAGG_RAW_*) --------------------------------------
# struct packet of packetparser (conntrack.c:34-49) and of dropreason (drop_reason.c:39-54)
RAW_PACKET_DTYPE = np.dtype({
    "names": ["t_nsec", "bytes", "src_ip", "dst_ip", "src_port", "dst_port", "seq", "ack_num",
              "tsval", "tsecr", "obs", "tdir", "proto", "flags", "is_reply", "pad",
              "bytes_fwd", "bytes_rep", "pkts_fwd", "pkts_rep"],
    "formats": ["<u8", "<u4", "<u4", "<u4", "<u2", "<u2", "<u4", "<u4", "<u4", "<u4",
                "u1", "u1", "u1", "u1", "u1", ("u1", 3), "<u8", "<u8", "<u4", "<u4"],
    "offsets": [0, 8, 12, 16, 20, 22, 24, 28, 32, 36, 40, 41, 42, 43, 44, 45, 48, 56, 64, 68],
    "itemsize": 72})
RAW_DROP_DTYPE = np.dtype({
    "names": ["src_ip", "dst_ip", "src_port", "dst_port", "skb_len", "return_val", "drop_type",
              "proto", "in_filtermap", "ts"],
    "formats": ["<u4", "<u4", "<u2", "<u2", "<u4", "<u4", "<u2", "u1", "u1", "<u8"],
    "offsets": [0, 4, 8, 10, 12, 16, 20, 22, 23, 24],
    "itemsize": 32})


def gen_raw_packets(n: int, pods: Pods, seed: int, *, pod_frac: float = 0.8, udp_frac: float = 0.10,
                    other_proto_frac: float = 0.02, odd_frac: float = 0.0,
                    out_of_range_frac: float = 0.0) -> np.ndarray:
    """n packetparser perf records (72 B each) as a uint8 buffer.  Fields the decode
    ignores (timestamps, TCP sequence/timestamp options, conntrack counters, padding)
    are random.  odd_frac: raw flag bytes with ECE/CWR bits, is_reply bytes other than
    0/1, observation points 4..255, traffic direction 0 or 3.  out_of_range_frac:
    traffic direction 4..255 (beyond the meta word; the eBPF program never emits it)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    r = np.zeros(n, RAW_PACKET_DTYPE)
    for f, hi in (("t_nsec", 1 << 62), ("seq", 1 << 32), ("ack_num", 1 << 32), ("tsval", 1 << 32),
                  ("tsecr", 1 << 32), ("bytes_fwd", 1 << 40), ("bytes_rep", 1 << 40),
                  ("pkts_fwd", 1 << 32), ("pkts_rep", 1 << 32)):
        r[f] = rng.integers(0, hi, n, dtype=np.uint64)
    r["pad"] = rng.integers(0, 256, (n, 3), dtype=np.uint8)
    r["src_ip"] = _pick_ips(rng, n, pods, pod_frac, None)
    r["dst_ip"] = _pick_ips(rng, n, pods, pod_frac, None)
    r["bytes"] = rng.integers(64, 1501, n, dtype=np.uint32)
    r["src_port"] = rng.integers(0, 1 << 16, n, dtype=np.uint32)
    r["dst_port"] = rng.integers(0, 1 << 16, n, dtype=np.uint32)
    pr = rng.random(n)
    proto = np.full(n, PROTO_TCP, np.uint8)
    proto[pr < udp_frac] = PROTO_UDP
    proto[(pr >= udp_frac) & (pr < udp_frac + other_proto_frac)] = PROTO_ICMP
    r["proto"] = proto
    r["obs"] = rng.integers(0, 4, n, dtype=np.uint8)
    r["tdir"] = rng.integers(1, 3, n, dtype=np.uint8)
    flags = FLAG_COMBOS[rng.integers(0, len(FLAG_COMBOS), n)].astype(np.uint8)
    r["flags"] = np.where(proto == PROTO_TCP, flags, np.uint8(1))  # UDP: always 1 (conntrack.c:46)
    r["is_reply"] = rng.integers(0, 2, n, dtype=np.uint8)
    if odd_frac:
        o = rng.random(n) < odd_frac
        k = rng.integers(0, 4, n)
        r["flags"] = np.where(o & (k == 0), rng.integers(0, 256, n, dtype=np.uint8), r["flags"])
        r["is_reply"] = np.where(o & (k == 1), rng.integers(2, 256, n, dtype=np.uint8), r["is_reply"])
        r["obs"] = np.where(o & (k == 2), rng.integers(4, 256, n, dtype=np.uint8), r["obs"])
        r["tdir"] = np.where(o & (k == 3), rng.choice(np.array([0, 3], np.uint8), n), r["tdir"])
    if out_of_range_frac:
        o = rng.random(n) < out_of_range_frac
        r["tdir"] = np.where(o, rng.integers(4, 256, n, dtype=np.uint8), r["tdir"])
    return r.view(np.uint8).reshape(-1)


def gen_raw_drops(n: int, pods: Pods, seed: int, *, pod_frac: float = 0.8, udp_frac: float = 0.2,
                  out_of_range_frac: float = 0.0) -> np.ndarray:
    """n dropreason perf records (32 B each) as a uint8 buffer; drop_type uniform over
    the drop_reason.h enum 0..6, or 8..65535 for out_of_range_frac of the rows."""
    rng = np.random.Generator(np.random.PCG64(seed))
    r = np.zeros(n, RAW_DROP_DTYPE)
    r["src_ip"] = _pick_ips(rng, n, pods, pod_frac, None)
    r["dst_ip"] = _pick_ips(rng, n, pods, pod_frac, None)
    r["src_port"] = rng.integers(0, 1 << 16, n, dtype=np.uint32)
    r["dst_port"] = rng.integers(0, 1 << 16, n, dtype=np.uint32)
    r["skb_len"] = rng.integers(40, 9001, n, dtype=np.uint32)
    r["return_val"] = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    r["drop_type"] = rng.integers(0, 7, n, dtype=np.uint16)
    r["proto"] = np.where(rng.random(n) < udp_frac, np.uint8(PROTO_UDP), np.uint8(PROTO_TCP))
    r["in_filtermap"] = rng.integers(0, 2, n, dtype=np.uint8)
    r["ts"] = rng.integers(0, 1 << 62, n, dtype=np.uint64)
    if out_of_range_frac:
        o = rng.random(n) < out_of_range_frac
        r["drop_type"] = np.where(o, rng.integers(8, 1 << 16, n, dtype=np.uint16), r["drop_type"])
    return r.view(np.uint8).reshape(-1)


def raw_packets_torch(src, dst, nbytes, meta, ports):
    """Device-side encoder for large batches: packetparser records whose decode yields
    the given columns (verdict FORWARDED, is_reply from meta bit 27, TCP flags from meta).
    Returns an int32 tensor [n, 18] (72-byte records) on the columns' device."""
    import torch
    n = src.shape[0]
    w = torch.zeros((n, 18), dtype=torch.int32, device=src.device)
    m = meta.to(torch.int64) & 0xFFFFFFFF
    p = ports.to(torch.int64) & 0xFFFFFFFF
    sp, dp = p & 0xFFFF, p >> 16
    sw = lambda x: ((x & 0xFF) << 8) | (x >> 8)  # noqa: E731 -- HostToNetShort is an involution
    proto, tdir, flags = m & 0xFF, (m >> 16) & 3, (m >> 21) & 0x3F
    w[:, 2] = nbytes
    w[:, 3] = src
    w[:, 4] = dst
    w[:, 5] = (sw(sp) | (sw(dp) << 16)).to(torch.int32)
    w[:, 10] = (2 | (tdir << 8) | (proto << 16) | (flags << 24)).to(torch.int32)  # obs 2
    w[:, 11] = ((m >> 27) & 1).to(torch.int32)
    return w


# ---- named configs ---------------------------------------------------------------------

LOCAL_FWD_DROP = [
    {"metric_name": "forward_count", "source_labels": ["namespace", "podname"]},
    {"metric_name": "forward_bytes", "source_labels": ["namespace", "podname"]},
    {"metric_name": "drop_count", "source_labels": ["namespace", "podname"]},
    {"metric_name": "drop_bytes", "source_labels": ["namespace", "podname"]},
]

C1_LABELS = ["ip", "namespace", "podname", "workload"]
C1_LOCAL = [{"metric_name": m, "source_labels": C1_LABELS}
            for m in ("forward_count", "forward_bytes", "drop_count", "drop_bytes")]
C1_REMOTE = [{"metric_name": m, "source_labels": C1_LABELS, "destination_labels": C1_LABELS}
             for m in ("forward_count", "forward_bytes", "drop_count", "drop_bytes")]

C5_SPEC = [
    {"metric_name": "tcp_flag_gauges", "source_labels": ["namespace", "podname"]},
    {"metric_name": "tcp_retransmission_count", "source_labels": ["namespace", "podname"]},
    {"metric_name": "dns_request_count", "source_labels": ["namespace", "podname"]},
    {"metric_name": "dns_response_count", "source_labels": ["namespace", "podname"]},
]

CONFIGS = {
    "c1": dict(records=1_000_000, pods=10_000, seed=1, gen={}),
    "c2": dict(records=100_000_000, pods=10_000, seed=2, gen={}),
    # C3: 5-tuples from 10^7 flows, src in the 10k pods, dst among 10^6 IPs
    "c3": dict(records=1 << 30, pods=10_000, seed=3, gen={"flows": 10_000_000, "n_dst": 1_000_000}),
    # C4: Zipf(1.2) 5-tuple ranks over 10^7 flows (so the flows' source and destination
    # pods are Zipf-skewed too: the hottest flow carries ~18 % of the records)
    "c4": dict(records=100_000_000, pods=10_000, seed=4,
               gen={"flows": 10_000_000, "flow_zipf": 1.2, "n_dst": 1_000_000}),
    # C4 through the remote context (C1_REMOTE: ip/namespace/podname/workload on both
    # sides): every update is a sparse group-by key, hot keys repeat within a wave, so this
    # is the contention case of the wave key de-duplication before the table's atomics
    "c4-remote": dict(records=100_000_000, pods=10_000, seed=4,
                      gen={"flows": 10_000_000, "flow_zipf": 1.2, "n_dst": 1_000_000}),
    # round-1 C4: Zipf(1.2) source pods only, independent destinations
    "c4-src": dict(records=100_000_000, pods=10_000, seed=4, gen={"zipf": 1.2}),
    "c5": dict(records=10_000_000, pods=100_000, seed=5,
               gen={"drop_frac": 0.0, "retrans_frac": 0.05, "dns_frac": 0.35}),
}


def gen_latency_records(n_conn: int, pods: Pods, api_ips: Sequence[int], seed: int = 0,
                        pairs: int = 4, background: int = 0, jitter: int = 8) -> Records:
    """Node <-> apiserver TCP traffic for the node-apiserver latency metrics (latency.go):
    n_conn connections (node IP, apiserver IP, random source port, 443), `pairs`
    request/reply exchanges each: TO_NETWORK requests carry TSval as tcp id, FROM_NETWORK
    replies carry it back as TSecr (packetparser_linux.go:622-628) 0.2-6 ms later; the
    first exchange is SYN / SYN+ACK.  Edge rows: 5 % unanswered requests, 3 % replies after
    the 500 ms TTL, 5 % repeated requests (same TSval), 2 % replies to no request.
    `background` pod-to-pod records (no tcp id or not apiserver traffic) are interleaved;
    records are in time order up to local swaps of `jitter` rows."""
    rng = np.random.Generator(np.random.PCG64(seed + 7000))
    u = np.uint32
    nodes = np.array([ip_le(10, 240, i >> 8, i & 255) for i in range(1, 33)], u)
    apis = np.asarray(api_ips, u)
    rows = []  # (time, src, dst, sport, dport, obs, flags, tcp_id)
    t0 = 1_700_000_000_000_000_000 + int(rng.integers(0, 10**9))
    SYN, ACK, PSH = 2, 16, 8
    for c in range(n_conn):
        node, api = int(rng.choice(nodes)), int(rng.choice(apis))
        sport = int(rng.integers(32768, 61000))
        t = t0 + int(rng.integers(0, 3 * 10**9))
        ts = int(rng.integers(1, 2**31))
        for k in range(pairs):
            t += int(rng.integers(1_000_000, 200_000_000))
            ts += int(rng.integers(1, 1000))
            rf, pf = (SYN, SYN | ACK) if k == 0 else (ACK | PSH, ACK)
            x = rng.random()
            rows.append((t, node, api, sport, 443, 3, rf, ts))
            if x < 0.05:
                continue  # unanswered
            if x < 0.10:  # the same request again (not stored twice, latency.go:268-275)
                rows.append((t + int(rng.integers(10_000, 900_000)), node, api, sport, 443, 3, rf, ts))
            lat = 600_000_000 if x > 0.97 else int(rng.integers(200_000, 6_000_000))
            rows.append((t + lat, api, node, 443, sport, 2, pf, ts))
            if x < 0.02:
                rows.append((t + lat + 1000, api, node, 443, sport, 2, pf, ts + 99_999))
    tmax = max(r[0] for r in rows)
    for _ in range(background):
        a, b = rng.integers(0, len(pods.ips), 2)
        obs = int(rng.integers(0, 4))
        rows.append((int(rng.integers(t0, tmax)), int(pods.ips[a]), int(pods.ips[b]),
                     int(rng.integers(1024, 65535)), 80, obs, ACK, int(rng.integers(0, 2)) * int(rng.integers(1, 2**31))))
    rows.sort(key=lambda r: r[0])
    for i in range(0, len(rows) - 1, 2):  # local disorder: the clock is a running max
        if rng.random() < 0.3 and jitter:
            j = min(len(rows) - 1, i + int(rng.integers(1, jitter)))
            rows[i], rows[j] = rows[j], rows[i]
    n = len(rows)
    time_ns = np.array([r[0] for r in rows], np.uint64)
    src = np.array([r[1] for r in rows], u)
    dst = np.array([r[2] for r in rows], u)
    ports = np.array([r[3] | (r[4] << 16) for r in rows], u)
    obs = np.array([r[5] for r in rows], u)
    flags = np.array([r[6] for r in rows], u)
    tcp_id = np.array([r[7] for r in rows], u)
    meta = pack_meta(np.full(n, 6, u), np.full(n, 1, u), np.where(obs == 3, 2, 1), 0, flags, obs=obs)
    return Records(src, dst, np.full(n, 100, u), meta, ports, np.zeros(n, u), [], tcp_id, time_ns)


def gen_latency_burst(n_req: int, api_ips: Sequence[int], seed: int = 0, spacing_ns: int = 1000,
                      reply_frac: float = 0.5, touch_frac: float = 0.05, background: int = 0) -> Records:
    """A burst of node -> apiserver requests outstanding at once (the ttlcache capacity,
    latency.go:35,120-121): n_req TO_NETWORK requests with distinct keys `spacing_ns`
    apart, a `reply_frac` share answered 0.2-300 ms later (early requests of a burst past
    the capacity were evicted, so their replies find nothing), and a `touch_frac` share
    repeated 400 ms later (same TSval: the Get hit touches the entry) and answered 650 ms
    after the first packet -- alive only through the touch.  Time-ordered records."""
    rng = np.random.Generator(np.random.PCG64(seed + 9100))
    u = np.uint32
    apis = np.asarray(api_ips, u)
    t0 = 1_700_000_000_000_000_000 + int(rng.integers(0, 10**9))
    ACK, PSH, SYN = 16, 8, 2
    rows = []
    node = np.array([ip_le(10, 241, i >> 8, i & 255) for i in range(1, 65)], u)
    for i in range(n_req):
        t = t0 + i * spacing_ns
        src, dst = int(node[i % len(node)]), int(apis[i % len(apis)])
        sport, ts = 1024 + (i * 7919) % 60000, 1 + i
        fl = SYN if i % 3 == 0 else ACK | PSH
        rows.append((t, src, dst, sport, 443, 3, fl, ts))
        x = rng.random()
        if x < touch_frac:
            rows.append((t + 400_000_000, src, dst, sport, 443, 3, fl, ts))
            rows.append((t + 650_000_000, dst, src, 443, sport, 2, SYN | ACK if fl == SYN else ACK, ts))
        elif x < touch_frac + reply_frac:
            rows.append((t + int(rng.integers(200_000, 300_000_000)), dst, src, 443, sport, 2,
                         SYN | ACK if fl == SYN else ACK, ts))
    tmax = max(r[0] for r in rows)
    for _ in range(background):
        rows.append((int(rng.integers(t0, tmax)), int(node[0]), int(node[1]), 5000, 80, 3, ACK, 0))
    rows.sort(key=lambda r: r[0])
    n = len(rows)
    time_ns = np.array([r[0] for r in rows], np.uint64)
    src = np.array([r[1] for r in rows], u)
    dst = np.array([r[2] for r in rows], u)
    ports = np.array([r[3] | (r[4] << 16) for r in rows], u)
    obs = np.array([r[5] for r in rows], u)
    flags = np.array([r[6] for r in rows], u)
    tcp_id = np.array([r[7] for r in rows], u)
    meta = pack_meta(np.full(n, 6, u), np.full(n, 1, u), np.where(obs == 3, 2, 1), 0, flags, obs=obs)
    return Records(src, dst, np.full(n, 100, u), meta, ports, np.zeros(n, u), [], tcp_id, time_ns)
