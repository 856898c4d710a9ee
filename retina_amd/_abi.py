"""ctypes declarations of ``include/gpuagg.h`` (the C-ABI boundary).

This is the binding a maintainer would add on the Python side; the Go side's cgo
binding is in ``go/pkg/gpuagg``.  Loading fails loudly when the
in-tree library is missing: there is no CPU fallback behind this ABI.
"""

from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPUAGG_LIB") or os.path.join(HERE, "libgpuagg.so")

ABI_VERSION = 3
OK, EINVAL, ENOMEM, EDEVICE, ECAPACITY, ESTATE, EDUPLICATE, ERANGE, ENOTFOUND = 0, -1, -2, -3, -4, -5, -6, -7, -8
ERR_NAMES = {EINVAL: "EINVAL", ENOMEM: "ENOMEM", EDEVICE: "EDEVICE", ECAPACITY: "ECAPACITY",
             ESTATE: "ESTATE", EDUPLICATE: "EDUPLICATE", ERANGE: "ERANGE", ENOTFOUND: "ENOTFOUND"}

u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)


class Config(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("device", C.c_int32), ("remote_context", C.c_int32),
                ("max_slots", C.c_uint32), ("max_ips", C.c_uint32),
                ("sparse_capacity_log2", C.c_uint32), ("cms_depth", C.c_uint32),
                ("cms_width_log2", C.c_uint32), ("hll_precision", C.c_uint32),
                ("flags", C.c_uint32), ("wide_list_mib", C.c_uint32), ("latency_limit", C.c_uint32)]
FLAG_NO_LDS_IP_TABLE = 1
FLAG_FOLD_PER_BATCH = 8  # diagnostics: fold the lists after every batch
FLAG_NO_HOT_KEYS = 16  # diagnostics: no LDS hot-key cache in front of the group-by table
FLAG_LDS_CUCKOO = 64  # diagnostics: cuckoo LDS IP image even when the radix image fits
FLAG_NO_WIDE_LISTS = 32  # diagnostics: wide group-by keys with memory-side atomics, no segment lists
FLAG_CPU_BACKEND = 128  # host threads and host memory instead of a device (GPUAGG_FLAG_CPU_BACKEND)
FLAG_ROW_RADIX = 256  # diagnostics: radix LDS IP images with the row table even when dense ones fit
FLAG_NARROW_ENTRIES = 512  # 24-byte wide-list entries when the plan's keys have no port / DNS fields


class MetricOptions(C.Structure):
    _fields_ = [("metric_name", C.c_char_p),
                ("source_labels", C.POINTER(C.c_char_p)), ("n_source_labels", C.c_uint32),
                ("source_labels_set", C.c_int32),
                ("destination_labels", C.POINTER(C.c_char_p)), ("n_destination_labels", C.c_uint32),
                ("destination_labels_set", C.c_int32)]


class Columns(C.Structure):
    _fields_ = [("src_ip", u32p), ("dst_ip", u32p), ("bytes", u32p), ("meta", u32p),
                ("ports", u32p), ("dns_id", u32p), ("tcp_id", u32p), ("time_ns", u64p)]


class Batch(C.Structure):
    _fields_ = [("cols", Columns), ("capacity", C.c_size_t)]


class StateDesc(C.Structure):
    _fields_ = [("dense_count", C.c_void_p), ("dense_len", C.c_size_t),
                ("dense_bytes", C.c_void_p),
                ("cms", C.c_void_p), ("cms_len", C.c_size_t),
                ("hll", C.c_void_p), ("hll_len", C.c_size_t),
                ("sparse_entry_words", C.c_size_t), ("sparse_len", C.c_size_t),
                ("latency", C.c_void_p), ("latency_len", C.c_size_t)]


class HubbleCols(C.Structure):
    _fields_ = [("src_identity", u32p), ("dst_identity", u32p), ("src_meta", u32p), ("dst_meta", u32p),
                ("summary_kind", u32p), ("summary_arg", u32p)]


class LatencyState(C.Structure):
    _fields_ = [("enabled", C.c_uint32), ("latency_buckets", C.c_uint64 * 11), ("latency_count", C.c_uint64),
                ("latency_sum", C.c_int64), ("handshake_buckets", C.c_uint64 * 11),
                ("handshake_count", C.c_uint64), ("handshake_sum", C.c_int64), ("no_response", C.c_uint64),
                ("pending", C.c_uint64), ("peak_pending", C.c_uint64), ("peak_live", C.c_uint64),
                ("capacity_evictions", C.c_uint64), ("capacity_batches", C.c_uint64), ("limit", C.c_uint64)]


class Stats(C.Structure):
    _fields_ = [("records", C.c_uint64), ("batches", C.c_uint64), ("sparse_entries", C.c_uint64),
                ("sparse_dropped", C.c_uint64), ("kernel_launches", C.c_uint64),
                ("kernel_ms", C.c_double), ("fold_ms", C.c_double), ("last_kernel", C.c_uint32),
                ("decoded", C.c_uint64), ("decode_out_of_range", C.c_uint64),
                ("decode_launches", C.c_uint64), ("decode_ms", C.c_double),
                ("sketch_launches", C.c_uint64), ("sketch_ms", C.c_double),
                ("async_returns", C.c_uint64)]


RAW_PACKET, RAW_DROP = 1, 2          # GPUAGG_RAW_* (include/gpuagg.h)
RECORD = 3  # GPUAGG_RECORD: decoded records, struct gpuagg_record (40 bytes)
RAW_SIZE = {RAW_PACKET: 72, RAW_DROP: 32, RECORD: 40}
FEED_HOST_DECODE, FEED_RAW_DMA = 0, 1  # GPUAGG_FEED_* (gpuagg_raw_feed_configure)
FEED_DRY_RUN = 0x100  # or'ed into a mode: stagings counted, never submitted (diagnostics)
LAT_SUM_WORDS = 35  # gpuagg_state_desc.latency: words [0, 35) sum, the rest max (gpuagg.h)


KERNEL_NAMES = {0: None, 1: "aggregate_kernel", 2: "dense_local_kernel", 3: "dense_lds_kernel", 4: "cpu"}


# (name, restype, argtypes) for every entry point declared in include/gpuagg.h
SIGNATURES = [
    ("gpuagg_create", C.c_int, [C.POINTER(Config), C.POINTER(C.c_void_p)]),
    ("gpuagg_destroy", None, [C.c_void_p]),
    ("gpuagg_last_error", C.c_char_p, [C.c_void_p]),
    ("gpuagg_reconcile", C.c_int, [C.c_void_p, C.POINTER(MetricOptions), C.c_size_t]),
    ("gpuagg_slot_intern", C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
                                     C.POINTER(C.c_int32)]),
    ("gpuagg_set_endpoints", C.c_int, [C.c_void_p, u32p, C.POINTER(C.c_int32), C.c_size_t, C.c_uint64]),
    ("gpuagg_dns_intern", C.c_int, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_char_p, C.c_char_p,
                                    C.c_uint32, u32p]),
    ("gpuagg_dns_retire", C.c_int, [C.POINTER(C.c_void_p), C.c_size_t, u32p, C.c_size_t,
                                    C.POINTER(C.c_size_t)]),
    ("gpuagg_alloc_batch", C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.POINTER(Batch))]),
    ("gpuagg_free_batch", None, [C.c_void_p, C.POINTER(Batch)]),
    ("gpuagg_submit", C.c_int, [C.c_void_p, C.POINTER(Batch), C.c_size_t]),
    ("gpuagg_submit_device", C.c_int, [C.c_void_p, C.POINTER(Columns), C.c_size_t]),
    ("gpuagg_decode_device", C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.POINTER(Columns)]),
    ("gpuagg_submit_raw_device", C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]),
    ("gpuagg_submit_raw", C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]),
    ("gpuagg_sync", C.c_int, [C.c_void_p]),
    ("gpuagg_reset", C.c_int, [C.c_void_p]),
    ("gpuagg_snapshot", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    ("gpuagg_result_count", C.c_size_t, [C.c_void_p]),
    ("gpuagg_result_series", C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_char_p),
                                       C.POINTER(C.c_uint32), C.POINTER(C.POINTER(C.c_char_p)),
                                       C.POINTER(C.POINTER(C.c_char_p)), C.POINTER(C.c_uint64)]),
    ("gpuagg_result_free", None, [C.c_void_p]),
    ("gpuagg_sketch_refresh", C.c_int, [C.c_void_p]),
    ("gpuagg_cms_estimate", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.POINTER(C.c_uint64)]),
    ("gpuagg_hll_estimate", C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_double)]),
    ("gpuagg_cms_copy", C.c_int, [C.c_void_p, u32p, C.c_size_t]),
    ("gpuagg_hll_copy", C.c_int, [C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t]),
    ("gpuagg_state", C.c_int, [C.c_void_p, C.POINTER(StateDesc)]),
    ("gpuagg_sparse_export", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("gpuagg_sparse_import", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("gpuagg_get_stats", C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    ("gpuagg_set_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("gpuagg_stream", C.c_void_p, [C.c_void_p]),
    ("gpuagg_kernel_name", C.c_char_p, [C.c_void_p]),
    ("gpuagg_sketch_kernel_name", C.c_char_p, [C.c_void_p]),
    ("gpuagg_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("gpuagg_build_id", C.c_char_p, []),
    ("gpuagg_shard_raw", C.c_int, [C.c_int, C.c_void_p, C.c_size_t, C.c_uint32, u32p]),
    ("gpuagg_shard_columns", C.c_int, [u32p, u32p, u32p, u32p, C.c_size_t, C.c_uint32, u32p]),
    ("gpuagg_cache_update_endpoint", C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
                                               u32p, C.c_size_t]),
    ("gpuagg_cache_delete_endpoint", C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p]),
    ("gpuagg_cache_update_service", C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p, C.c_uint32]),
    ("gpuagg_cache_delete_service", C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p]),
    ("gpuagg_cache_update_node", C.c_int, [C.c_void_p, C.c_char_p, C.c_uint32]),
    ("gpuagg_cache_delete_node", C.c_int, [C.c_void_p, C.c_char_p]),
    ("gpuagg_cache_commit", C.c_int, [C.c_void_p, C.c_uint64]),
    ("gpuagg_retire_slots", C.c_int, [C.c_void_p, C.POINTER(C.c_size_t)]),
    ("gpuagg_merge", C.c_int, [C.POINTER(C.c_void_p), C.c_size_t]),
    ("gpuagg_result_family", C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p)]),
    ("gpuagg_result_dropped", C.c_uint64, [C.c_void_p]),
    ("gpuagg_result_render_text", C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("gpuagg_result_text", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    ("gpuagg_set_apiserver_ips", C.c_int, [C.c_void_p, u32p, C.c_size_t]),
    ("gpuagg_latency_read", C.c_int, [C.c_void_p, C.POINTER(LatencyState)]),
    ("gpuagg_set_time_offset", C.c_int, [C.c_void_p, C.c_int64]),
    ("gpuagg_ipcache_set", C.c_int, [C.c_void_p, u32p, u32p, u32p, C.c_size_t]),
    ("gpuagg_hubble_decode_device", C.c_int, [C.c_void_p, C.POINTER(Columns), C.c_size_t,
                                              C.POINTER(HubbleCols)]),
    ("gpuagg_enrich_device", C.c_int, [C.c_void_p, C.POINTER(Columns), C.c_size_t, C.c_void_p, C.c_void_p]),
    ("gpuagg_submit_enrich", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]),
    ("gpuagg_raw_feed_create", C.c_int, [C.POINTER(C.c_void_p), C.c_size_t, C.c_int, C.c_size_t,
                                         C.POINTER(C.c_void_p)]),
    ("gpuagg_raw_feed_configure", C.c_int, [C.c_void_p, C.c_uint32, C.c_int]),
    ("gpuagg_raw_feed_put", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("gpuagg_raw_feed_flush", C.c_int, [C.c_void_p]),
    ("gpuagg_raw_feed_submitted", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t]),
    ("gpuagg_raw_feed_destroy", None, [C.c_void_p]),
]

_lib = None


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load the in-tree engine library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError("retina_amd: %s is missing; run __graft_entry__.build() "
                          "(there is no CPU fallback)" % path)
    # One HIP runtime per process.  torch 2.10+rocm ships its own libamdhip64.so and
    # libhsa-runtime64.so (torch/lib, SONAMEs libamdhip64.so.7 / libhsa-runtime64.so.1)
    # and its libraries NEED them by the unversioned names.  libgpuagg.so NEEDs
    # libamdhip64.so.7: loaded AFTER torch, the dynamic linker matches that SONAME to
    # torch's copy and the process has one runtime; loaded BEFORE torch, it maps
    # /opt/rocm/lib's copy, torch's NEEDED "libamdhip64.so" matches no loaded name and a
    # second runtime is mapped -- whose HIP init then finds no GPU ("No HIP GPUs are
    # available", round-1 smoke).  So torch is imported first, and the result is checked.
    import torch  # noqa: F401
    lib = C.CDLL(path)
    # (only libamdhip64 is enforced: under rocprofv3 the profiler's own tool library maps
    # /opt/rocm's libhsa-runtime64 beside torch's, by design)
    runtimes = hip_runtimes_mapped()
    if len(runtimes.get("libamdhip64", ())) > 1:
        raise ImportError("retina_amd: two HIP runtimes are mapped in this process: %r" % runtimes)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def hip_runtimes_mapped() -> dict:
    """{"libamdhip64": {paths}, "libhsa-runtime64": {paths}} mapped in this process."""
    out = {}
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.split()[-1] if len(line.split()) >= 6 else ""
                base = os.path.basename(path)
                for stem in ("libamdhip64", "libhsa-runtime64"):
                    if base.startswith(stem + ".so"):
                        out.setdefault(stem, set()).add(os.path.realpath(path))
    except OSError:
        pass
    return out
