"""ctypes wrapper of oracle/ref_cpu.c (TEST INFRASTRUCTURE ONLY: tests + bench cpu_baseline)."""

from __future__ import annotations

import ctypes as C
import os
import subprocess
import time
from typing import Dict, List, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "ref_cpu.c")
LIB = os.path.join(HERE, "libref_cpu.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        tmp = "%s.%d.tmp" % (LIB, os.getpid())
        subprocess.run(["gcc", "-O2", "-std=c11", "-D_GNU_SOURCE", "-shared", "-fPIC", "-Wall", "-pthread",
                        "-o", tmp, SRC], check=True)
        os.replace(tmp, LIB)  # atomic: concurrent builders (spawned ranks) never see a partial file
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB)
        L.ref_create.restype = C.c_void_p
        L.ref_create.argtypes = [C.c_int]
        L.ref_add_metric.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_char_p), C.c_int, C.c_int,
                                     C.POINTER(C.c_char_p), C.c_int, C.c_int]
        L.ref_add_endpoint.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
                                       C.POINTER(C.c_uint32), C.c_int]
        L.ref_add_dns.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_char_p, C.c_char_p, C.c_uint32]
        u = C.POINTER(C.c_uint32)
        L.ref_process.argtypes = [C.c_void_p, u, u, u, u, u, u, C.c_size_t]
        L.ref_process_tuned.argtypes = [C.c_void_p, u, u, u, u, u, u, C.c_size_t, C.c_int]
        L.ref_finish.restype = C.c_size_t
        L.ref_finish.argtypes = [C.c_void_p]
        L.ref_series.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                 C.POINTER(C.c_uint64)]
        L.ref_destroy.argtypes = [C.c_void_p]
        _lib = L
    return _lib


class RefCPU:
    h = None  # set once ref_create succeeds; close()/__del__ check it

    def __init__(self, spec: List[dict], endpoints, remote: bool, dns=()):
        L = lib()
        self.L = L
        self.h = L.ref_create(1 if remote else 0)
        keep = []

        def arr(lst):
            if lst is None:
                return None, 0, 0
            a = (C.c_char_p * max(1, len(lst)))(*[s.encode() for s in lst])
            keep.append(a)
            return a, len(lst), 1
        for s in spec:
            a, na, sa = arr(s.get("source_labels"))
            b, nb, sb = arr(s.get("destination_labels"))
            if L.ref_add_metric(self.h, s["metric_name"].encode(), a, na, sa, b, nb, sb) != 0:
                raise ValueError("reference would panic on metric %s" % s["metric_name"])
        for e in endpoints:
            ips = np.ascontiguousarray(np.asarray(e.ips, np.uint32))
            owner = e.owner_refs[0] if e.owner_refs else None
            L.ref_add_endpoint(self.h, e.namespace.encode(), e.name.encode(),
                               owner[0].encode() if owner else None,
                               owner[1].encode() if owner else None,
                               ips.ctypes.data_as(C.POINTER(C.c_uint32)), len(ips))
        for p in dns:
            L.ref_add_dns(self.h, p.rcode, ",".join(p.qtypes).encode(), p.query.encode(),
                          ",".join(p.ips).encode(), p.num_answers)

    def process(self, recs) -> float:
        u = C.POINTER(C.c_uint32)
        cols = [np.ascontiguousarray(getattr(recs, k), np.uint32)
                for k in ("src_ip", "dst_ip", "bytes", "meta", "ports", "dns_id")]
        t0 = time.perf_counter()
        rc = self.L.ref_process(self.h, *[c.ctypes.data_as(u) for c in cols], len(cols[0]))
        dt = time.perf_counter() - t0
        if rc != 0:
            raise ValueError("ref_process failed")
        return dt

    def process_tuned(self, recs, threads: int) -> float:
        """Tuned mode: integer keys, `threads` threads, per-thread tables merged at the end."""
        u = C.POINTER(C.c_uint32)
        cols = [np.ascontiguousarray(getattr(recs, k), np.uint32)
                for k in ("src_ip", "dst_ip", "bytes", "meta", "ports", "dns_id")]
        t0 = time.perf_counter()
        rc = self.L.ref_process_tuned(self.h, *[c.ctypes.data_as(u) for c in cols], len(cols[0]), threads)
        dt = time.perf_counter() - t0
        if rc != 0:
            raise ValueError("ref_process_tuned failed")
        return dt

    def series(self) -> Dict[Tuple[str, Tuple[str, ...]], int]:
        n = self.L.ref_finish(self.h)
        out = {}
        m = C.c_char_p()
        lab = C.c_char_p()
        v = C.c_uint64()
        for i in range(n):
            self.L.ref_series(self.h, i, C.byref(m), C.byref(lab), C.byref(v))
            vals = tuple(lab.value.decode().split("\x1f")[1:]) if lab.value else ()
            out[("networkobservability_" + m.value.decode(), vals)] = v.value
        return out

    def close(self):
        if self.h:
            self.L.ref_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def values_only(series) -> Dict[Tuple[str, Tuple[str, ...]], int]:
    """Engine/oracle series keyed by (metric, label values) for comparison with RefCPU."""
    return {(k[0], tuple(v for _, v in k[1])): val for k, val in series.items()}
