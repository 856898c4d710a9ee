"""Multi-GPU sharding and merge: one process per GPU.

* Records are sharded by a seeded 64-bit hash of the 5-tuple, so every flow's
  records land on one rank (the path's per-record updates are independent; only the
  accumulated state needs an exchange).
* The per-epoch merge is one collective per state kind over torch.distributed
  (backend "nccl" = RCCL over xGMI on MI355X, "gloo" in CPU tests):
    dense counters  all_reduce SUM (u64, carried as int64: two's complement == mod 2^64)
    count-min       all_reduce SUM (u32 carried as int32)
    HLL registers   all_reduce MAX (u8)
    sparse table    all_gather of compacted (k0,k1,k2,count,bytes) entries, inserted-and-
                    added on the merging rank (gpuagg_sparse_import)
    latency         all_reduce SUM of the histogram / count / sum / no_response words
  Counters and count-min are linear and HLL max is exact, so the merged state equals the
  1-GPU state bit for bit.
"""

from __future__ import annotations

from typing import List, Optional

import numpy as np

from . import _abi

_U64 = np.uint64
_M1, _M2 = _U64(0xff51afd7ed558ccd), _U64(0xc4ceb9fe1a85ec53)
SHARD_SEED = _U64(0x1F2E3D4C5B6A7988)


def _fmix64(k: np.ndarray) -> np.ndarray:
    k = k.astype(_U64, copy=True)
    with np.errstate(over="ignore"):
        k ^= k >> _U64(33)
        k *= _M1
        k ^= k >> _U64(33)
        k *= _M2
        k ^= k >> _U64(33)
    return k


def shard_of(src_ip, dst_ip, ports, meta, world: int) -> np.ndarray:
    """Rank owning each record: h(direction-free 5-tuple) mod world.  The two (ip, port)
    ends are ordered before hashing, so a request and its reply (mirrored 5-tuples) land
    on one rank, which the node-apiserver latency join needs (latency.go:256-305)."""
    p = ports.astype(_U64)
    a = (src_ip.astype(_U64) << _U64(16)) | (p & _U64(0xFFFF))
    b = (dst_ip.astype(_U64) << _U64(16)) | (p >> _U64(16))
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    proto = (meta.astype(_U64) & _U64(0xFF)) << _U64(48)
    h = _fmix64(lo ^ _fmix64(hi ^ proto ^ SHARD_SEED))
    return (h % _U64(world)).astype(np.int64)


def shard_records(recs, world: int, rank: int):
    """This rank's records (a workloads.Records-like object with numpy columns)."""
    own = shard_of(recs.src_ip, recs.dst_ip, recs.ports, recs.meta, world) == rank
    out = type(recs)(*(getattr(recs, k)[own] for k in ("src_ip", "dst_ip", "bytes", "meta",
                                                        "ports", "dns_id")), recs.dns)
    for k in ("tcp_id", "time_ns"):
        if getattr(recs, k, None) is not None:
            setattr(out, k, getattr(recs, k)[own])
    return out


# ---- collectives over torch tensors (device views on GPU, CPU tensors under gloo) -------

def merge_dense(cnt, byt, group=None) -> None:
    import torch.distributed as dist
    dist.all_reduce(cnt, group=group)
    dist.all_reduce(byt, group=group)


def merge_cms(cms, group=None) -> None:
    import torch.distributed as dist
    dist.all_reduce(cms, group=group)


def merge_hll(hll, group=None) -> None:
    import torch.distributed as dist
    dist.all_reduce(hll, op=dist.ReduceOp.MAX, group=group)


def gather_entries(entries, n: int, dst: int = 0, group=None) -> Optional[List]:
    """All-gathers variable-length (n, 5) int64 entry blocks; returns them on `dst`."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    cnt = torch.tensor([n], dtype=torch.int64, device=entries.device)
    sizes = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(sizes, cnt, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes) if sizes else 0
    pad = torch.zeros((max(m, 1), 5), dtype=torch.int64, device=entries.device)
    if n:
        pad[:n] = entries[:n]
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    if dist.get_rank(group) != dst:
        return None
    return [o[:s] for o, s in zip(outs, sizes)]


def merge_entries_host(blocks) -> dict:
    """Host-side restatement of import: sum count/bytes of equal (k0,k1,k2) keys."""
    out = {}
    for b in blocks:
        for row in b.tolist():
            k = (row[0] & 0xFFFFFFFFFFFFFFFF, row[1] & 0xFFFFFFFFFFFFFFFF, row[2] & 0xFFFFFFFFFFFFFFFF)
            c, v = out.get(k, (0, 0))
            out[k] = (c + row[3], v + row[4])
    return out


class _CAI:
    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}


def device_view(ptr: int, n: int, typestr: str, device):
    """torch tensor aliasing engine-owned device memory (no copy)."""
    import torch
    return torch.as_tensor(_CAI(ptr, n, typestr), device=device)


_HOST_CTYPES = {"<i8": np.int64, "<i4": np.int32, "|u1": np.uint8}


def host_view(ptr: int, n: int, typestr: str):
    """torch tensor aliasing engine-owned HOST memory (the CPU backend's state; no copy)."""
    import ctypes
    import torch
    dt = np.dtype(_HOST_CTYPES[typestr])
    buf = (ctypes.c_uint8 * (n * dt.itemsize)).from_address(ptr)
    return torch.from_numpy(np.frombuffer(buf, dtype=dt, count=n))


def merge_engine(engine, group=None, dst: int = 0) -> None:
    """Per-epoch merge of a GpuAgg's state across ranks: rank `dst` ends with the node
    total, every other rank is reset (gpuagg_reset) so the next epoch counts only new
    records.

    Backend "nccl" (RCCL over xGMI) reduces the engine's device memory in place through
    __cuda_array_interface__ views.  Backend "gloo" (CPU tests, and several ranks sharing
    one GPU) stages each array through host memory: copy out, reduce, copy back.  An
    engine on the CPU backend (GPUAGG_FLAG_CPU_BACKEND) keeps its state in host memory,
    which gloo reduces in place."""
    import torch
    import torch.distributed as dist
    on_cpu = bool(engine.cfg.flags & _abi.FLAG_CPU_BACKEND)
    device = torch.device("cpu") if on_cpu else torch.device("cuda", engine.device)
    on_host = dist.get_backend(group) == "gloo"
    if on_cpu and not on_host:
        raise ValueError("merge_engine: a CPU-backend engine merges over gloo")
    dev_sync = (lambda: None) if on_cpu else (lambda: torch.cuda.synchronize(device))
    engine.sync()
    st = engine.state()
    me = dist.get_rank(group)

    def reduce(ptr, n, typestr, op):
        if on_cpu:
            dist.reduce(host_view(ptr, n, typestr), dst, op=op, group=group)
            return
        view = device_view(ptr, n, typestr, device)
        if not on_host:
            dist.reduce(view, dst, op=op, group=group)
            return
        h = view.cpu()
        dist.reduce(h, dst, op=op, group=group)
        if me == dst:
            view.copy_(h)

    if st.dense_len:
        reduce(st.dense_count, st.dense_len, "<i8", dist.ReduceOp.SUM)
        reduce(st.dense_bytes, st.dense_len, "<i8", dist.ReduceOp.SUM)
    if st.cms_len:
        reduce(st.cms, st.cms_len, "<i4", dist.ReduceOp.SUM)
    if st.hll_len:
        reduce(st.hll, st.hll_len, "|u1", dist.ReduceOp.MAX)
    # node-apiserver latency histograms / counts / sums and no_response: summed like the
    # counters (the pending requests stay on their shard: each shard runs its own clock)
    if st.latency_len:  # words [0, LAT_SUM_WORDS) summed, the rest (peak live) max-merged
        reduce(st.latency, _abi.LAT_SUM_WORDS, "<i8", dist.ReduceOp.SUM)
        reduce(st.latency + 8 * _abi.LAT_SUM_WORDS, st.latency_len - _abi.LAT_SUM_WORDS, "<i8",
               dist.ReduceOp.MAX)
    # sparse table: every rank's compact entries gathered on dst and inserted-and-added
    cap = int(st.sparse_len)
    local = torch.empty((max(cap, 1), 5), dtype=torch.int64, device=device)
    # the engine writes on its own stream: nothing of torch's may still be pending on
    # this memory (a zero-fill racing the export was seen to wipe exported rows)
    dev_sync()
    n = engine.sparse_export(local.data_ptr(), cap) if cap else 0
    dev_sync()
    blocks = gather_entries(local.cpu() if on_host else local, n, dst, group)
    if blocks is not None:
        for r, b in enumerate(blocks):
            if r != me and b.shape[0]:
                b = b.to(device).contiguous()
                dev_sync()
                engine.sparse_import(b.data_ptr(), int(b.shape[0]))
    engine.sync()
    dev_sync()
    if me != dst:
        engine.reset()
