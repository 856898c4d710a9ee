"""N>1 path on CPU: 5-tuple sharding + the per-epoch merge collectives, world_size 2 over
gloo (127.0.0.1).  Each rank builds its shard's state with the CPU restatements; the merged
state must equal the single-process state bit for bit (SURVEY.md 8e invariant)."""

import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from retina_amd import dist as D
from retina_amd import workloads as W


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import sketch as S
        from oracle.ref_cpu import RefCPU
        from oracle.vectorized import LocalDense
        pods = W.make_pods(300, seed=5)
        recs = W.gen_records(40_000, pods, seed=5, drop_frac=0.1, retrans_frac=0.05, udp_frac=0.2)
        mine = D.shard_records(recs, world, rank)
        # dense counters: sum
        spec = W.LOCAL_FWD_DROP + [{"metric_name": "tcp_flag_gauges", "source_labels": ["podname"]}]
        v = LocalDense(spec, pods.endpoints)
        v.add(mine)
        arrs = [torch.from_numpy(a.view(np.int64).copy()) for a in (v.fwd_c, v.fwd_b, v.drop_c, v.drop_b, v.flag_c)]
        D.merge_dense(arrs[0], arrs[1])   # forward count / bytes
        D.merge_dense(arrs[2], arrs[3])   # drop count / bytes
        dist.all_reduce(arrs[4])          # tcp flags
        # count-min: sum; HLL: max
        cms = np.zeros((4, 1 << 10), np.uint32)
        S.cms_update(cms, mine.src_ip, mine.dst_ip, mine.ports, mine.meta & np.uint32(0xFF))
        tc = torch.from_numpy(cms.view(np.int32).copy())
        D.merge_cms(tc)
        ips = {int(ip): s for s, e in enumerate(pods.endpoints) for ip in e.ips}
        slot = np.array([ips.get(int(x), -1) for x in mine.src_ip], np.int64)
        hll = np.zeros((len(pods.endpoints), 1 << 8), np.uint8)
        S.hll_update(hll, slot, mine.dst_ip, 8)
        th = torch.from_numpy(hll.copy())
        D.merge_hll(th)
        # sparse entries: all_gather to rank 0, host merge (restates gpuagg_sparse_import)
        r = RefCPU(W.C1_REMOTE, pods.endpoints, True)
        r.process(mine)
        ser = r.series()
        rows = []
        for (m, vals), val in ser.items():
            h = int.from_bytes(hashlib.blake2b(repr((m, vals)).encode(), digest_size=8).digest(), "little")
            rows.append([h & 0x7FFFFFFFFFFFFFFF, len(vals), 0, val, 0])
        keys = {(row[0], row[1], 0): (m, vals) for row, ((m, vals), _) in zip(rows, ser.items())}
        ent = torch.tensor(rows or [[0] * 5], dtype=torch.int64)
        blocks = D.gather_entries(ent, len(rows), 0)
        gathered_keys = [None] * world
        dist.all_gather_object(gathered_keys, keys)
        out = None
        if rank == 0:
            merged = D.merge_entries_host(blocks)
            allk = {}
            for kk in gathered_keys:
                allk.update(kk)
            out = {allk[k]: c for k, (c, _) in merged.items()}
        q.put((rank, [a.numpy().copy() for a in arrs], tc.numpy().copy(), th.numpy().copy(), out))
    finally:
        dist.destroy_process_group()


def test_two_rank_merge_equals_single():
    from oracle import sketch as S
    from oracle.ref_cpu import RefCPU
    from oracle.vectorized import LocalDense
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    # A fresh container can take minutes on each spawned rank's first `import torch`, so
    # poll with a long overall deadline and fail fast only if a rank actually died.
    import queue
    import time
    res = {}
    deadline = time.monotonic() + 900
    while len(res) < world:
        try:
            rank, arrs, cms, hll, sparse = q.get(timeout=10)
            res[rank] = (arrs, cms, hll, sparse)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"gloo rank exited with {dead}"
            assert time.monotonic() < deadline, "gloo ranks did not report within 900 s"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    pods = W.make_pods(300, seed=5)
    recs = W.gen_records(40_000, pods, seed=5, drop_frac=0.1, retrans_frac=0.05, udp_frac=0.2)
    # the shards partition the records
    own = D.shard_of(recs.src_ip, recs.dst_ip, recs.ports, recs.meta, world)
    assert set(np.unique(own)) <= {0, 1} and 0 < (own == 0).sum() < len(recs)
    spec = W.LOCAL_FWD_DROP + [{"metric_name": "tcp_flag_gauges", "source_labels": ["podname"]}]
    v = LocalDense(spec, pods.endpoints)
    v.add(recs)
    want = [a.view(np.int64) for a in (v.fwd_c, v.fwd_b, v.drop_c, v.drop_b, v.flag_c)]
    cms = np.zeros((4, 1 << 10), np.uint32)
    S.cms_update(cms, recs.src_ip, recs.dst_ip, recs.ports, recs.meta & np.uint32(0xFF))
    ips = {int(ip): s for s, e in enumerate(pods.endpoints) for ip in e.ips}
    slot = np.array([ips.get(int(x), -1) for x in recs.src_ip], np.int64)
    hll = np.zeros((len(pods.endpoints), 1 << 8), np.uint8)
    S.hll_update(hll, slot, recs.dst_ip, 8)
    r = RefCPU(W.C1_REMOTE, pods.endpoints, True)
    r.process(recs)
    want_sparse = r.series()
    for rank in range(world):
        arrs, c, h, _ = res[rank]
        for a, w in zip(arrs, want):
            assert np.array_equal(a, w)
        assert np.array_equal(c.view(np.uint32), cms)
        assert np.array_equal(h, hll)
    assert res[0][3] == want_sparse


def test_shard_of_is_direction_free():
    """A request and its reply (mirrored 5-tuples) land on one rank (the latency join)."""
    rng = np.random.default_rng(5)
    n = 10_000
    s, d = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32), rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    sp, dp = rng.integers(0, 65536, n).astype(np.uint32), rng.integers(0, 65536, n).astype(np.uint32)
    meta = np.full(n, 6, np.uint32)
    for world in (2, 8):
        a = D.shard_of(s, d, sp | (dp << np.uint32(16)), meta, world)
        b = D.shard_of(d, s, dp | (sp << np.uint32(16)), meta, world)
        assert np.array_equal(a, b) and len(np.unique(a)) == world
