"""Diagnostic (GPU box): where do group-by entries differ -- the kernel inserts of the
sharded engines, or the export/import merge?  Prints one JSON line per check."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from retina_amd import GpuAgg, dist as D, workloads as W  # noqa: E402
from tests.helpers import make_engine, to_device  # noqa: E402

SPEC = W.LOCAL_FWD_DROP + W.C5_SPEC


def entries(g):
    st = g.state()
    buf = torch.zeros((max(1, st.sparse_len), 5), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    n = g.sparse_export(buf.data_ptr(), st.sparse_len)
    out = {}
    for row in buf[:n].cpu().numpy().tolist():
        k = (row[0] & (2**64 - 1), row[1] & (2**64 - 1), row[2] & (2**64 - 1))
        c, b = out.get(k, (0, 0))
        out[k] = (c + row[3], b + row[4])
    return out, buf, n


def main():
    kw = dict(cms_depth=4, cms_width_log2=16, hll_precision=10) if os.environ.get("DIAG_SKETCH") else {}
    print(json.dumps({"sketch": bool(kw)}), flush=True)
    pods = W.make_pods(1_500, seed=21)
    recs = W.gen_records(1_500_000, pods, seed=21, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.1,
                         udp_frac=0.15, n_queries=3_000)
    one = make_engine(pods, SPEC, False, 0, recs, sparse_capacity_log2=21, **kw)
    one.submit_device(GpuAgg.device_columns(*to_device(recs, 0)), len(recs))
    one.sync()
    want, _, _ = entries(one)
    parts = []
    for r in range(2):
        g = make_engine(pods, SPEC, False, 0, recs, sparse_capacity_log2=21, **kw)
        sh = D.shard_records(recs, 2, r)
        g.submit_device(GpuAgg.device_columns(*to_device(sh, 0)), len(sh))
        g.sync()
        parts.append(g)
    ea, _, _ = entries(parts[0])
    eb, bufb, nb = entries(parts[1])
    hs = dict(ea)
    for k, (c, b) in eb.items():
        c0, b0 = hs.get(k, (0, 0))
        hs[k] = (c0 + c, b0 + b)
    print(json.dumps({"check": "shards_sum_vs_single", "equal": hs == want, "n_want": len(want),
                      "n_sum": len(hs), "diff": sum(1 for k in set(hs) | set(want) if hs.get(k) != want.get(k)),
                      "total_want": sum(c for c, _ in want.values()), "total_sum": sum(c for c, _ in hs.values()),
                      "dropped": [p.stats()["sparse_dropped"] for p in parts]}), flush=True)
    parts[0].sparse_import(bufb.data_ptr(), nb)
    parts[0].sync()
    em, _, _ = entries(parts[0])
    print(json.dumps({"check": "import_vs_host_sum", "equal": em == hs, "n": len(em),
                      "diff": sum(1 for k in set(hs) | set(em) if hs.get(k) != em.get(k)),
                      "total": sum(c for c, _ in em.values())}), flush=True)
    # single-engine determinism: a second identical engine
    two = make_engine(pods, SPEC, False, 0, recs, sparse_capacity_log2=21, **kw)
    two.submit_device(GpuAgg.device_columns(*to_device(recs, 0)), len(recs))
    two.sync()
    w2, _, _ = entries(two)
    print(json.dumps({"check": "single_repeat", "equal": w2 == want,
                      "diff": sum(1 for k in set(w2) | set(want) if w2.get(k) != want.get(k))}), flush=True)


if __name__ == "__main__":
    main()
