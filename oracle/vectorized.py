"""numpy restatement of local-context, endpoint-keyed metrics at full batch sizes
(TEST INFRASTRUCTURE ONLY).

Covers forward / drop / tcpflags / tcpretrans with options among namespace, podname,
workload, service -- the groups whose label values depend only on the endpoint.  It
restates getLocalCtxValues (types.go:379-416: src -> egress, dst -> ingress, nil and
apiserver endpoints skipped) and the per-metric update rules (forward.go:197-224,
drops.go:363-395, tcpflags.go:111-175, tcpretrans.go:281-298) as bincounts, so a
100M-record batch can be checked exactly in seconds.  Pinned against oracle.py by
tests/test_ref_cpu.py.
"""

from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import oracle as O

FLAG_NAMES = ["FIN", "SYNACK", "SYN", "ACK", "RST", "PSH", "URG"]


def _slots(ips: np.ndarray, table_ips: np.ndarray, table_slot: np.ndarray) -> np.ndarray:
    order = np.argsort(table_ips)
    ti, ts = table_ips[order], table_slot[order]
    pos = np.searchsorted(ti, ips)
    pos = np.minimum(pos, len(ti) - 1)
    hit = ti[pos] == ips
    return np.where(hit, ts[pos], -1)


def _flag_bits(flags: np.ndarray) -> List[np.ndarray]:
    fin, syn, rst, psh, ack, urg = [(flags >> i) & 1 for i in range(6)]
    synack = syn & ack
    return [fin, synack, syn & (1 - ack), ack & (1 - syn), rst, psh, urg]


class LocalDense:
    """Accumulates per-(slot, side, sub) counts for one local-context spec."""

    def __init__(self, spec: Sequence[dict], endpoints):
        self.spec = list(spec)
        self.endpoints = endpoints
        ip_owner = {}
        for s, e in enumerate(endpoints):
            for ip in e.ips:
                ip_owner[int(ip)] = s  # later endpoints own shared IPs (cache.go:204-233)
        self.table_ips = np.fromiter(ip_owner.keys(), np.uint32, len(ip_owner))
        self.table_slot = np.fromiter(ip_owner.values(), np.int64, len(ip_owner))
        self.api = np.array([e.namespace == O.APISERVER_ENDPOINT_NAME and e.name == O.APISERVER_ENDPOINT_NAME
                             for e in endpoints])
        ns = len(endpoints)
        self.ns = ns
        z = lambda k: np.zeros((ns, 2, k), np.uint64)  # noqa: E731
        self.fwd_c, self.fwd_b = z(1), z(1)
        self.drop_c, self.drop_b = z(8), z(8)
        self.flag_c = z(7)
        self.ret_c = z(1)

    def add(self, recs) -> None:
        ss = _slots(recs.src_ip, self.table_ips, self.table_slot)
        ds = _slots(recs.dst_ip, self.table_ips, self.table_slot)
        meta = recs.meta
        proto = meta & 0xFF
        verdict = (meta >> 8) & 0xFF
        verdict = np.where(verdict == 0, 1, verdict)
        reason = ((meta >> 18) & 7).astype(np.int64)
        flags = (meta >> 21) & 0x3F
        nb = recs.bytes.astype(np.uint64)
        for side, slot in ((0, ds), (1, ss)):  # 0 ingress (destination), 1 egress (source)
            ok = slot >= 0
            ok &= ~self.api[np.where(ok, slot, 0)]
            sl = np.where(ok, slot, 0)

            def bc(mask, idx_sub, nsub, w=None):
                m = ok & mask
                key = sl[m] * nsub + idx_sub[m]
                return np.bincount(key, weights=None if w is None else w[m].astype(np.float64),
                                   minlength=self.ns * nsub)

            zero = np.zeros(len(sl), np.int64)
            fwd = verdict == 1
            self.fwd_c[:, side, 0] += bc(fwd, zero, 1).astype(np.uint64)
            self.fwd_b[:, side, 0] += self._exact_sum(sl, ok & fwd, nb, zero, 1)
            drp = verdict == 2
            self.drop_c[:, side, :] += bc(drp, reason, 8).reshape(self.ns, 8).astype(np.uint64)
            self.drop_b[:, side, :] += self._exact_sum(sl, ok & drp, nb, reason, 8).reshape(self.ns, 8)
            tcpf = fwd & (proto == 6)
            for k, bits in enumerate(_flag_bits(flags)):
                self.flag_c[:, side, k] += bc(tcpf & (bits == 1), zero, 1).astype(np.uint64)
            self.ret_c[:, side, 0] += bc(verdict == 15, zero, 1).astype(np.uint64)

    def _exact_sum(self, sl, mask, w, sub, nsub) -> np.ndarray:
        """Exact uint64 sums (bincount weights are float64: fine below 2^53 per bin)."""
        key = sl[mask] * nsub + sub[mask]
        s = np.bincount(key, weights=w[mask].astype(np.float64), minlength=self.ns * nsub)
        assert s.max(initial=0) < 2 ** 53
        return s.astype(np.uint64)

    def series(self) -> Dict[Tuple[str, Tuple[Tuple[str, str], ...]], int]:
        """Series exist for every touched key, also with value 0 (Add(0) creates one)."""
        out: Dict = {}

        def put(metric, names, values, count, value):
            if count:
                k = (O.RETINA_NAMESPACE + "_" + metric, tuple(zip(names, values)))
                out[k] = out.get(k, 0) + int(value)

        for s in self.spec:
            name = s["metric_name"]
            opts = O.ContextOptions(s.get("source_labels"), O.CTX_LOCAL)
            ln = opts.get_labels()
            if not ln:
                continue
            is_flags = "tcp" in name and "flag" in name.lower() and "retrans" not in name.lower()
            is_retrans = "tcp" in name and "retrans" in name.lower()
            for slot in range(self.ns):
                e = self.endpoints[slot]
                wl = [O.Workload(*e.owner_refs[0])] if e.owner_refs else None
                vals = opts.get_by_direction_values(O.Flow(source=O.Endpoint(e.namespace, e.name, workloads=wl)), False)
                for side, d in ((0, "ingress"), (1, "egress")):
                    if name == "forward_count":
                        put("adv_forward_count", ["direction"] + ln, [d] + vals, self.fwd_c[slot, side, 0], self.fwd_c[slot, side, 0])
                    elif name == "forward_bytes":
                        put("adv_forward_bytes", ["direction"] + ln, [d] + vals, self.fwd_c[slot, side, 0], self.fwd_b[slot, side, 0])
                    elif name in ("drop_count", "drop_bytes"):
                        for r in range(8):
                            c = self.drop_c[slot, side, r]
                            put("adv_" + name, ["reason", "direction"] + ln,
                                [O.enum_string(O.DROP_REASON_NAMES, r), d] + vals, c,
                                c if name == "drop_count" else self.drop_b[slot, side, r])
                    elif is_flags:
                        for f in range(7):
                            c = self.flag_c[slot, side, f]
                            put("adv_tcpflags_count", ["flag"] + ln, [FLAG_NAMES[f]] + vals, c, c)
                    elif is_retrans:
                        c = self.ret_c[slot, side, 0]
                        put("adv_tcpretrans_count", ["direction"] + ln, [d] + vals, c, c)
        return out
