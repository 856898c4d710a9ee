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


def pack_meta(proto, verdict, tdir=0, reason=0, flags=0, is_reply=0, dns_type=0):
    """meta word of include/gpuagg.h (vectorised over numpy arrays)."""
    u = np.uint32
    return (np.asarray(proto, u) & u(0xFF)) | ((np.asarray(verdict, u) & u(0xFF)) << u(8)) \
        | ((np.asarray(tdir, u) & u(3)) << u(16)) | ((np.asarray(reason, u) & u(7)) << u(18)) \
        | ((np.asarray(flags, u) & u(0x3F)) << u(21)) | ((np.asarray(is_reply, u) & u(1)) << u(27)) \
        | ((np.asarray(dns_type, u) & u(3)) << u(28))


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


def gen_records(n: int, pods: Pods, seed: int, *, pod_frac: float = 0.8, drop_frac: float = 0.10,
                retrans_frac: float = 0.0, dns_frac: float = 0.0, udp_frac: float = 0.0,
                other_proto_frac: float = 0.0, zipf: Optional[float] = None,
                n_queries: int = 100_000, odd_frac: float = 0.0) -> Records:
    """Vectorised record generator (SURVEY.md 8d distributions).

    odd_frac adds edge rows: unknown / out-of-range traffic directions, verdicts no
    metric consumes, drop reason 7, destination 255.255.255.255."""
    rng = np.random.Generator(np.random.PCG64(seed))
    u = np.uint32
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
    return Records(src, dst, nbytes, meta.astype(u), (sport | (dport << u(16))).astype(u), dns_id,
                   payloads)


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
    "c3": dict(records=1 << 30, pods=10_000, seed=3, gen={}),
    "c4": dict(records=100_000_000, pods=10_000, seed=4, gen={"zipf": 1.2}),
    "c5": dict(records=10_000_000, pods=100_000, seed=5,
               gen={"drop_frac": 0.0, "retrans_frac": 0.05, "dns_frac": 0.35}),
}
