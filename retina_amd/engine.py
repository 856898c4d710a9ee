"""Python host of the flow-aggregation engine (over the C-ABI in include/gpuagg.h).

Mirrors the reference's host-side vocabulary so tests read like Retina's own:

* ``GpuAgg.reconcile(context_options)``  -- Module.Reconcile / updateMetricsContexts
  (pkg/module/metrics/metrics_module.go:205-264)
* ``GpuAgg.set_endpoints`` / ``load_endpoints`` -- the enricher's IP cache snapshot
  (pkg/controllers/cache/cache.go:110-233)
* ``GpuAgg.submit`` / ``submit_device``    -- Enricher.Write of a whole batch
  (pkg/enricher/enricher.go:185-187)
* ``GpuAgg.snapshot``                      -- what the AdvancedRegistry would expose
  (pkg/exporter/prometheusexporter.go:17-66)
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _abi

SeriesKey = Tuple[str, Tuple[Tuple[str, str], ...]]


class GpuAggError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("%s (%d): %s" % (_abi.ERR_NAMES.get(code, "E?"), code, msg))
        self.code = code


@dataclass
class ContextOptions:
    """crd MetricsContextOptions (metricsconfiguration_types.go:27-58); None = nil slice."""
    metric_name: str
    source_labels: Optional[List[str]] = None
    destination_labels: Optional[List[str]] = None


def _opts(o) -> ContextOptions:
    if isinstance(o, ContextOptions):
        return o
    if isinstance(o, dict):
        return ContextOptions(o["metric_name"], o.get("source_labels"), o.get("destination_labels"))
    return ContextOptions(o.metric_name, o.source_labels, o.destination_labels)


@dataclass
class Endpoint:
    """A pod's identity as the enricher copies it into flow.Endpoint (enricher.go:142-183)."""
    namespace: str
    name: str
    ips: Sequence[int]  # LE u32 IPv4, primary first (ipaddr.go:35-50)
    owner_refs: Optional[Sequence[Tuple[str, str]]] = None  # (kind, name)


class HostBatch:
    """A library-owned pinned batch with numpy views of its columns."""

    def __init__(self, ptr, capacity: int):
        self.ptr = ptr
        self.capacity = capacity
        cols = ptr.contents.cols
        for name in ("src_ip", "dst_ip", "bytes", "meta", "ports", "dns_id", "tcp_id", "time_ns"):
            p = getattr(cols, name)
            setattr(self, name, np.ctypeslib.as_array(p, shape=(capacity,)))

    def fill(self, batch, start: int = 0, n: Optional[int] = None) -> int:
        """Copy rows [start, start+n) of an object with numpy column attributes."""
        total = len(batch.src_ip)
        n = min(self.capacity, total - start) if n is None else n
        for name in ("src_ip", "dst_ip", "bytes", "meta", "ports", "dns_id", "tcp_id", "time_ns"):
            src = getattr(batch, name, None)
            if src is not None:
                getattr(self, name)[:n] = src[start:start + n]
            else:
                getattr(self, name)[:n] = 0
        return n


class GpuAgg:
    """One engine context bound to one MI355X (gfx950) device."""

    def __init__(self, device: int = 0, remote_context: bool = False, max_slots: int = 1 << 14,
                 max_ips: int = 1 << 16, sparse_capacity_log2: int = 22, cms_depth: int = 0,
                 cms_width_log2: int = 20, hll_precision: int = 0, flags: int = 0,
                 wide_list_mib: int = 0, latency_limit: int = 0):
        self.lib = _abi.load()
        cfg = _abi.Config(_abi.ABI_VERSION, device, 1 if remote_context else 0, max_slots, max_ips,
                          sparse_capacity_log2, cms_depth, cms_width_log2 if cms_depth else 0,
                          hll_precision, flags, wide_list_mib, latency_limit)
        h = C.c_void_p()
        rc = self.lib.gpuagg_create(C.byref(cfg), C.byref(h))
        if rc != _abi.OK:
            raise GpuAggError(rc, "gpuagg_create failed (device %d; a gfx950 GPU is required)" % device)
        self.h = h
        self.cfg = cfg
        self.device = device
        self.remote_context = remote_context
        self._batches: List[HostBatch] = []

    # -- plumbing --------------------------------------------------------------------
    def _check(self, rc: int) -> None:
        if rc != _abi.OK:
            msg = self.lib.gpuagg_last_error(self.h)
            raise GpuAggError(rc, msg.decode() if msg else "")

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.gpuagg_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- Module.Reconcile ------------------------------------------------------------
    def reconcile(self, context_options: Iterable) -> None:
        opts = [_opts(o) for o in context_options]
        keep = []

        def strarr(lst):
            if lst is None:
                return None, 0, 0
            arr = (C.c_char_p * max(1, len(lst)))(*[s.encode() for s in lst])
            keep.append(arr)
            return arr, len(lst), 1

        arr = (_abi.MetricOptions * max(1, len(opts)))()
        for i, o in enumerate(opts):
            s, ns, sset = strarr(o.source_labels)
            d, nd, dset = strarr(o.destination_labels)
            arr[i].metric_name = o.metric_name.encode()
            arr[i].source_labels = C.cast(s, C.POINTER(C.c_char_p)) if s is not None else None
            arr[i].n_source_labels = ns
            arr[i].source_labels_set = sset
            arr[i].destination_labels = C.cast(d, C.POINTER(C.c_char_p)) if d is not None else None
            arr[i].n_destination_labels = nd
            arr[i].destination_labels_set = dset
        self._check(self.lib.gpuagg_reconcile(self.h, arr, len(opts)))

    # -- endpoints / dictionaries ----------------------------------------------------
    def slot_intern(self, namespace: str, pod: str, workload_kind: Optional[str] = None,
                    workload_name: Optional[str] = None) -> int:
        s = C.c_int32()
        self._check(self.lib.gpuagg_slot_intern(
            self.h, namespace.encode(), pod.encode(),
            None if workload_kind is None else workload_kind.encode(),
            None if workload_name is None else (workload_name or "").encode(), C.byref(s)))
        return s.value

    def set_endpoints(self, ips: np.ndarray, slots: np.ndarray, version: int = 0) -> None:
        ips = np.ascontiguousarray(ips, dtype=np.uint32)
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        self._check(self.lib.gpuagg_set_endpoints(
            self.h, ips.ctypes.data_as(_abi.u32p), slots.ctypes.data_as(C.POINTER(C.c_int32)),
            len(ips), version))

    def load_endpoints(self, endpoints: Sequence[Endpoint], version: int = 0) -> None:
        """Cache.UpdateRetinaEndpoint for every endpoint in order, then installs the
        cache's IP -> pod map (cache.go:196-233: a later endpoint that takes an IP of an
        earlier one deletes that whole earlier endpoint)."""
        for ep in endpoints:
            self.cache_update_endpoint(ep)
        self.cache_commit(version)

    # -- the IP cache (cache.go), natively in the engine ---------------------------------
    def cache_update_endpoint(self, ep: Endpoint) -> None:
        owner = ep.owner_refs[0] if ep.owner_refs else None
        ips = np.ascontiguousarray(np.asarray(list(ep.ips), dtype=np.uint32))
        self._check(self.lib.gpuagg_cache_update_endpoint(
            self.h, ep.namespace.encode(), ep.name.encode(),
            None if owner is None else owner[0].encode(),
            None if owner is None else (owner[1] or "").encode(),
            ips.ctypes.data_as(_abi.u32p), len(ips)))

    def cache_delete_endpoint(self, namespace: str, name: str) -> None:
        self._check(self.lib.gpuagg_cache_delete_endpoint(self.h, namespace.encode(), name.encode()))

    def cache_update_service(self, namespace: str, name: str, ip: int) -> None:
        self._check(self.lib.gpuagg_cache_update_service(self.h, namespace.encode(), name.encode(), ip))

    def cache_delete_service(self, namespace: str, name: str) -> None:
        self._check(self.lib.gpuagg_cache_delete_service(self.h, namespace.encode(), name.encode()))

    def cache_update_node(self, name: str, ip: int) -> None:
        self._check(self.lib.gpuagg_cache_update_node(self.h, name.encode(), ip))

    def cache_delete_node(self, name: str) -> None:
        self._check(self.lib.gpuagg_cache_delete_node(self.h, name.encode()))

    def cache_commit(self, version: int = 0) -> None:
        self._check(self.lib.gpuagg_cache_commit(self.h, version))

    def retire_slots(self) -> int:
        """Frees the slots the installed IP table no longer references (epoch boundary)."""
        n = C.c_size_t()
        self._check(self.lib.gpuagg_retire_slots(self.h, C.byref(n)))
        return n.value

    def merge_from(self, others: Sequence["GpuAgg"]) -> None:
        """gpuagg_merge: fold the state of `others` (any devices) into this engine and
        reset them -- the single-process multi-GPU epoch merge."""
        arr = (C.c_void_p * (1 + len(others)))(self.h, *[o.h for o in others])
        self._check(self.lib.gpuagg_merge(arr, len(arr)))

    def dns_intern(self, rcode: int, qtypes: Sequence[str], query: str, ips: Sequence[str],
                   num_answers: int) -> int:
        out = C.c_uint32()
        self._check(self.lib.gpuagg_dns_intern(self.h, rcode, ",".join(qtypes).encode(),
                                               query.encode(), ",".join(ips).encode(),
                                               num_answers, C.byref(out)))
        self._dns_hwm = max(getattr(self, "_dns_hwm", 0), out.value + 1)  # ids < hwm
        return out.value

    def dns_retire(self, others: Sequence["GpuAgg"] = ()) -> List[int]:
        """gpuagg_dns_retire over this engine and `others` (one dictionary interned alike on
        each): the DNS ids no group-by key references any more, now free for reuse."""
        ctxs = [self] + list(others)
        arr = (C.c_void_p * len(ctxs))(*[e.h for e in ctxs])
        cap = max(1, getattr(self, "_dns_hwm", 0))  # every id ever handed out is below it
        ids = (C.c_uint32 * cap)()
        n = C.c_size_t()
        self._check(self.lib.gpuagg_dns_retire(arr, len(ctxs), ids, cap, C.byref(n)))
        return list(ids[:n.value])

    # -- records -----------------------------------------------------------------------

    def alloc_batch(self, capacity: int) -> HostBatch:
        p = C.POINTER(_abi.Batch)()
        self._check(self.lib.gpuagg_alloc_batch(self.h, capacity, C.byref(p)))
        b = HostBatch(p, capacity)
        self._batches.append(b)
        return b

    def submit(self, batch: HostBatch, n: int) -> None:
        self._check(self.lib.gpuagg_submit(self.h, batch.ptr, n))

    def submit_enrich(self, batch: HostBatch, n: int):
        """gpuagg_submit + the batch's enriched endpoints (src, dst slot arrays, -1: none)."""
        src = np.empty(n, np.int32)
        dst = np.empty(n, np.int32)
        self._check(self.lib.gpuagg_submit_enrich(self.h, batch.ptr, n, src.ctypes.data, dst.ctypes.data))
        return src, dst

    def submit_numpy(self, batch, chunk: int = 1 << 22) -> None:
        """Host-fed path: streams a numpy column batch through pinned buffers."""
        total = len(batch.src_ip)
        hb = None
        for b in self._batches:
            if b.capacity >= min(chunk, max(total, 1)):
                hb = b
                break
        if hb is None:
            hb = self.alloc_batch(max(1, min(chunk, total)))
        start = 0
        while start < total:
            n = hb.fill(batch, start)
            self.submit(hb, n)
            start += n

    @staticmethod
    def device_columns(src_ip, dst_ip, nbytes, meta, ports=None, dns_id=None, tcp_id=None,
                       time_ns=None) -> "_abi.Columns":
        """Columns from device tensors (torch int32/uint32, contiguous, on this device).

        The engine reads them on its own HIP stream, which does not wait for torch's: the
        device is synchronised here so every pending write to the tensors has landed."""
        import torch
        torch.cuda.synchronize(src_ip.device)

        def ptr(t):
            if t is None:
                return None
            return C.cast(C.c_void_p(t.data_ptr()), _abi.u32p)
        t = None if time_ns is None else C.cast(C.c_void_p(time_ns.data_ptr()), _abi.u64p)
        return _abi.Columns(ptr(src_ip), ptr(dst_ip), ptr(nbytes), ptr(meta), ptr(ports), ptr(dns_id),
                            ptr(tcp_id), t)

    # -- node-apiserver latency (gpuagg_latency.hip) ----------------------------------
    def set_apiserver_ips(self, ips: Sequence[int]) -> None:
        arr = (C.c_uint32 * max(1, len(ips)))(*[int(x) for x in ips])
        self._check(self.lib.gpuagg_set_apiserver_ips(self.h, arr, len(ips)))

    def set_time_offset(self, ns: int) -> None:
        self._check(self.lib.gpuagg_set_time_offset(self.h, int(ns)))

    def latency_state(self) -> dict:
        st = _abi.LatencyState()
        self._check(self.lib.gpuagg_latency_read(self.h, C.byref(st)))
        return {"enabled": st.enabled, "latency_buckets": list(st.latency_buckets),
                "latency_count": st.latency_count, "latency_sum": st.latency_sum,
                "handshake_buckets": list(st.handshake_buckets), "handshake_count": st.handshake_count,
                "handshake_sum": st.handshake_sum, "no_response": st.no_response, "pending": st.pending,
                "peak_pending": st.peak_pending, "peak_live": st.peak_live,
                "capacity_evictions": st.capacity_evictions, "capacity_batches": st.capacity_batches,
                "limit": st.limit}

    # -- enriched-flow emission, standard mode (enrich_kernel) --------------------------
    def enrich_device(self, cols: "_abi.Columns", n: int, src_slot, dst_slot) -> None:
        """Enricher.enrich + export (enricher.go:102-140) for n device-resident records:
        writes each record's source / destination pod slot (-1: no endpoint) into the two
        int32 device tensors; async on the engine's stream (sync() waits)."""
        self._torch_sync()
        for t in (src_slot, dst_slot):
            if t.numel() < n or t.element_size() != 4:
                raise ValueError("enrich_device: output tensors need n int32 elements")
        self._check(self.lib.gpuagg_enrich_device(self.h, C.byref(cols), n, C.c_void_p(src_slot.data_ptr()),
                                                  C.c_void_p(dst_slot.data_ptr())))

    # -- Hubble-mode L3/L4 enrichment (gpuagg_hubble.hip) ------------------------------
    def ipcache_set(self, ips: Sequence[int], identities: Sequence[int], meta_ids: Sequence[int]) -> None:
        n = len(ips)
        arr = lambda v: (C.c_uint32 * max(1, n))(*[int(x) for x in v])  # noqa: E731
        self._check(self.lib.gpuagg_ipcache_set(self.h, arr(ips), arr(identities), arr(meta_ids), n))

    def hubble_decode_device(self, cols: "_abi.Columns", n: int, out) -> None:
        """out: six device tensors (int32): src/dst identity, src/dst meta, summary kind, arg."""
        self._torch_sync()

        def ptr(t):
            return C.cast(C.c_void_p(t.data_ptr()), _abi.u32p)
        hc = _abi.HubbleCols(*[ptr(t) for t in out])
        self._check(self.lib.gpuagg_hubble_decode_device(self.h, C.byref(cols), n, C.byref(hc)))

    def submit_device(self, cols: "_abi.Columns", n: int) -> None:
        self._check(self.lib.gpuagg_submit_device(self.h, C.byref(cols), n))

    # -- raw perf records (gpuagg_decode.hip) ----------------------------------------
    def _torch_sync(self) -> None:
        """Device memory handed over as raw pointers may have torch work pending on it
        (the CPU backend's buffers are host memory: nothing to wait for)."""
        if self.cfg.flags & _abi.FLAG_CPU_BACKEND:
            return
        import torch
        torch.cuda.synchronize(self.device)

    def decode_device(self, kind: int, raw_ptr: int, n: int, out: "_abi.Columns") -> None:
        """Decode n raw records (device pointer) into device columns, async."""
        self._torch_sync()
        self._check(self.lib.gpuagg_decode_device(self.h, kind, C.c_void_p(raw_ptr), n, C.byref(out)))

    def submit_raw_device(self, kind: int, raw_ptr: int, n: int) -> None:
        """Decode + aggregate n raw records already in this device's HBM, async."""
        self._torch_sync()
        self._check(self.lib.gpuagg_submit_raw_device(self.h, kind, C.c_void_p(raw_ptr), n))

    def submit_raw(self, kind: int, raw: np.ndarray, chunk: int = 1 << 22) -> None:
        """Host-fed raw records (a uint8 buffer of n * record-size bytes)."""
        size = _abi.RAW_SIZE[kind]
        raw = np.ascontiguousarray(raw).view(np.uint8).reshape(-1)
        if raw.size % size:
            raise ValueError("raw buffer is not a whole number of %d-byte records" % size)
        n = raw.size // size
        for a in range(0, n, chunk):
            m = min(chunk, n - a)
            part = raw[a * size:(a + m) * size]
            self._check(self.lib.gpuagg_submit_raw(self.h, kind, part.ctypes.data_as(C.c_void_p), m))

    def sync(self) -> None:
        self._check(self.lib.gpuagg_sync(self.h))

    def reset(self) -> None:
        self._check(self.lib.gpuagg_reset(self.h))

    # -- output ------------------------------------------------------------------------
    def snapshot_text(self) -> str:
        """The snapshot in the Prometheus text exposition format (gpuagg_result_text)."""
        r = C.c_void_p()
        self._check(self.lib.gpuagg_snapshot(self.h, C.byref(r)))
        try:
            n = C.c_size_t()
            p = C.c_void_p()
            self._check(self.lib.gpuagg_result_text(r, C.byref(p), C.byref(n)))
            return C.string_at(p.value, n.value).decode() if n.value else ""
        finally:
            self.lib.gpuagg_result_free(r)

    def snapshot_families(self) -> Dict[str, Tuple[str, str]]:
        """{metric: (prometheus type, help)} of the snapshot's series."""
        r = C.c_void_p()
        self._check(self.lib.gpuagg_snapshot(self.h, C.byref(r)))
        out = {}
        try:
            metric, t, h = C.c_char_p(), C.c_char_p(), C.c_char_p()
            for i in range(self.lib.gpuagg_result_count(r)):
                self._check(self.lib.gpuagg_result_series(r, i, C.byref(metric), None, None, None, None))
                self._check(self.lib.gpuagg_result_family(r, i, C.byref(t), C.byref(h)))
                out[metric.value.decode()] = (t.value.decode(), h.value.decode())
        finally:
            self.lib.gpuagg_result_free(r)
        return out

    def snapshot(self) -> Dict[SeriesKey, int]:
        r = C.c_void_p()
        self._check(self.lib.gpuagg_snapshot(self.h, C.byref(r)))
        out: Dict[SeriesKey, int] = {}
        self.last_dropped = 0
        try:
            self.last_dropped = int(self.lib.gpuagg_result_dropped(r))
            n = self.lib.gpuagg_result_count(r)
            metric = C.c_char_p()
            nl = C.c_uint32()
            names = C.POINTER(C.c_char_p)()
            vals = C.POINTER(C.c_char_p)()
            v = C.c_uint64()
            for i in range(n):
                self._check(self.lib.gpuagg_result_series(r, i, C.byref(metric), C.byref(nl),
                                                          C.byref(names), C.byref(vals), C.byref(v)))
                labels = tuple((names[j].decode(), vals[j].decode()) for j in range(nl.value))
                out[(metric.value.decode(), labels)] = v.value
        finally:
            self.lib.gpuagg_result_free(r)
        return out

    # -- sketches ----------------------------------------------------------------------
    def sketch_refresh(self) -> None:
        self._check(self.lib.gpuagg_sketch_refresh(self.h))

    def cms_estimate(self, src_ip: int, dst_ip: int, ports: int, proto: int) -> int:
        out = C.c_uint64()
        self._check(self.lib.gpuagg_cms_estimate(self.h, src_ip, dst_ip, ports, proto, C.byref(out)))
        return out.value

    def hll_estimate(self, slot: int) -> float:
        out = C.c_double()
        self._check(self.lib.gpuagg_hll_estimate(self.h, slot, C.byref(out)))
        return out.value

    def cms_array(self) -> np.ndarray:
        d = self.state()
        a = np.zeros(d.cms_len, np.uint32)
        self._check(self.lib.gpuagg_cms_copy(self.h, a.ctypes.data_as(_abi.u32p), a.size))
        return a.reshape(self.cfg.cms_depth, -1) if a.size else a

    def hll_array(self) -> np.ndarray:
        """HLL registers [slots covered, 2^p] (rows grow with the slots in use)."""
        d = self.state()
        a = np.zeros(d.hll_len, np.uint8)
        self._check(self.lib.gpuagg_hll_copy(self.h, a.ctypes.data_as(C.POINTER(C.c_uint8)), a.size))
        return a.reshape(-1, 1 << self.cfg.hll_precision) if a.size else a

    # -- merge / introspection -----------------------------------------------------------
    def state(self) -> "_abi.StateDesc":
        d = _abi.StateDesc()
        self._check(self.lib.gpuagg_state(self.h, C.byref(d)))
        return d

    def sparse_export(self, dev_ptr: int, cap: int) -> int:
        self._torch_sync()
        n = C.c_size_t()
        self._check(self.lib.gpuagg_sparse_export(self.h, C.c_void_p(dev_ptr), cap, C.byref(n)))
        return n.value

    def sparse_import(self, dev_ptr: int, n: int) -> None:
        self._torch_sync()
        self._check(self.lib.gpuagg_sparse_import(self.h, C.c_void_p(dev_ptr), n))

    def stats(self) -> Dict[str, float]:
        s = _abi.Stats()
        self._check(self.lib.gpuagg_get_stats(self.h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in _abi.Stats._fields_}

    def kernel_name(self) -> str:
        """Signature of the last launch's aggregation kernel (rocprofv3 spelling)."""
        return (self.lib.gpuagg_kernel_name(self.h) or b"").decode()

    def sketch_kernel_name(self) -> str:
        """The last sketch pass's kernels (rocprofv3 spelling, joined by "+")."""
        return (self.lib.gpuagg_sketch_kernel_name(self.h) or b"").decode()

    def set_timing(self, enabled: bool) -> None:
        self._check(self.lib.gpuagg_set_timing(self.h, 1 if enabled else 0))


# struct gpuagg_record (include/gpuagg.h): the Go plugin's Record, back to back
RECORD_DTYPE = np.dtype([("src_ip", "<u4"), ("dst_ip", "<u4"), ("bytes", "<u4"), ("meta", "<u4"),
                         ("ports", "<u4"), ("dns_id", "<u4"), ("tcp_id", "<u4"), ("pad_", "<u4"),
                         ("time_ns", "<u8")])


def records_aos(recs) -> np.ndarray:
    """W.Records (SoA) -> gpuagg_record array (AoS), as the Go plugin holds them."""
    n = len(recs.src_ip)
    a = np.zeros(n, RECORD_DTYPE)
    for k in ("src_ip", "dst_ip", "bytes", "meta", "ports", "dns_id"):
        a[k] = getattr(recs, k)
    if getattr(recs, "tcp_id", None) is not None:
        a["tcp_id"] = recs.tcp_id
    if getattr(recs, "time_ns", None) is not None:
        a["time_ns"] = recs.time_ns
    return a


class RawFeed:
    """Node-wide ingestion over one context per device (gpuagg_raw_feed_*): raw perf samples
    (kind RAW_PACKET / RAW_DROP) or decoded gpuagg_record arrays (RECORD) are sharded by the
    5-tuple (gpuagg_shard_raw's / gpuagg_shard_columns' function) and copied into each
    context's pinned staging in the library; full stagings are submitted as they fill."""

    def __init__(self, engines, kind: int, capacity: int = 1 << 20, threads: int = 0, mode: int = None):
        self.engines = list(engines)
        self.lib = self.engines[0].lib
        self.kind = kind
        self.size = _abi.RAW_SIZE[kind]
        arr = (C.c_void_p * len(self.engines))(*[e.h for e in self.engines])
        h = C.c_void_p()
        rc = self.lib.gpuagg_raw_feed_create(arr, len(self.engines), kind, capacity, C.byref(h))
        if rc != _abi.OK:
            msg = self.lib.gpuagg_last_error(self.engines[0].h)
            raise GpuAggError(rc, "gpuagg_raw_feed_create: %s" % (msg.decode() if msg else ""))
        self.h = h
        if threads or mode is not None:
            self.configure(threads, _abi.FEED_RAW_DMA if mode is None else mode)

    def configure(self, threads: int = 0, mode: int = _abi.FEED_RAW_DMA) -> None:
        """Host threads per put (0: keep) and, for raw kinds, where samples are decoded
        (FEED_RAW_DMA, the default: the 72/32-byte samples are copied and decoded on the
        GPU; FEED_HOST_DECODE: on the feed's threads, only the plan's columns cross PCIe)."""
        rc = self.lib.gpuagg_raw_feed_configure(self.h, threads, mode)
        if rc != _abi.OK:
            raise GpuAggError(rc, "gpuagg_raw_feed_configure")

    def put(self, raw: np.ndarray) -> None:
        raw = np.ascontiguousarray(raw).view(np.uint8).reshape(-1)
        if raw.size % self.size:
            raise ValueError("raw buffer is not a whole number of %d-byte records" % self.size)
        rc = self.lib.gpuagg_raw_feed_put(self.h, raw.ctypes.data_as(C.c_void_p), raw.size // self.size)
        if rc != _abi.OK:
            raise GpuAggError(rc, "gpuagg_raw_feed_put")

    def flush(self) -> None:
        rc = self.lib.gpuagg_raw_feed_flush(self.h)
        if rc != _abi.OK:
            raise GpuAggError(rc, "gpuagg_raw_feed_flush")

    def submitted(self) -> list:
        a = (C.c_uint64 * len(self.engines))()
        rc = self.lib.gpuagg_raw_feed_submitted(self.h, a, len(self.engines))
        if rc != _abi.OK:
            raise GpuAggError(rc, "gpuagg_raw_feed_submitted")
        return list(a)

    def close(self) -> None:
        if self.h:
            self.lib.gpuagg_raw_feed_destroy(self.h)
            self.h = None
