"""Simulation of one wide_kernel workgroup's LDS hot-key cache on the C4-remote bench stream
(2 / 3 / 4 candidate ways, 2^15-bit doorkeeper): list appends per record and the fullest
segment list.  Keys and hashes are stand-ins (flow tuple + meta), not the kernel's.
    PYTHONPATH=. python exp/r6/sim_hot_cache.py"""
import numpy as np
from retina_amd import workloads as W
pods = W.make_pods(10_000, seed=4)
n = 390_625
res = {}
for wg in range(4):
    r = W.gen_records(n, pods, seed=5000 + wg, **W.CONFIGS["c4"]["gen"])
    key = (r.src_ip.astype(np.uint64) << np.uint64(32)) | r.dst_ip.astype(np.uint64)
    key = key ^ (r.meta.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15))
    h = (key * np.uint64(0xff51afd7ed558ccd)) ^ (key >> np.uint64(29))
    h = h * np.uint64(0xc4ceb9fe1a85ec53); h = h ^ (h >> np.uint64(32))
    u, inv = np.unique(h, return_inverse=True)
    seg = ((h & np.uint64((1 << 24) - 1)) >> np.uint64(12)).astype(np.int64).tolist()
    invl = inv.tolist()
    db = ((h >> np.uint64(40)) & np.uint64((1 << 15) - 1)).astype(np.int64).tolist()
    for ncand in (2, 3, 4):
        hot_n = 2048
        cands = [((h + np.uint64(q * 0x9E37)) & np.uint64(hot_n - 1)).astype(np.int64).tolist() for q in range(ncand)]
        door = set(); tags = {}; app = np.zeros(4096, np.int64)
        for j in range(n):
            k = invl[j]; b = db[j]; claim = b in door; door.add(b)
            done = False
            for q in range(ncand):
                e = cands[q][j]
                tg = tags.get(e)
                if tg is None:
                    if not claim: continue
                    tags[e] = k; done = True; break
                if tg == k: done = True; break
            if not done: app[seg[j]] += 1
        for e, k in tags.items(): app[int((u[k] & np.uint64((1 << 24) - 1)) >> np.uint64(12))] += 1
        res.setdefault(ncand, []).append((app.sum() / n, app.max()))
for k, v in res.items(): print(k, v)
