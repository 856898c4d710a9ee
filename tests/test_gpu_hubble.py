"""Hubble-mode L3/L4 enrichment on the GPU (gpuagg_hubble.hip) against oracle/hubble.py,
record by record: identities, K8s metadata ids and summaries (rendered from the codes)."""

import numpy as np
import pytest

from oracle import hubble as H
from oracle import oracle as O
from oracle import records as R
from retina_amd import workloads as W

from .helpers import dns_dict, make_engine

pytestmark = pytest.mark.gpu


def test_hubble_decode_matches_oracle(gpu_device):
    import torch
    from retina_amd import GpuAgg
    pods = W.make_pods(500, seed=61)
    recs = W.gen_records(40_000, pods, seed=62, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.15, udp_frac=0.1,
                         n_queries=200, other_proto_frac=0.02)
    rng = np.random.default_rng(63)
    ips = pods.ips.tolist()
    keep = rng.random(len(ips)) < 0.9                      # 10 % of pod IPs not in the ipcache
    ident = rng.integers(256, 1 << 24, len(ips))
    ident[rng.random(len(ips)) < 0.05] = H.ID_HOST          # some reserved identities
    ident[rng.random(len(ips)) < 0.05] = H.ID_REMOTE_NODE
    meta_id = np.where(rng.random(len(ips)) < 0.8, np.arange(len(ips)), 0xFFFFFFFF)
    sel = np.nonzero(keep)[0]
    g = make_engine(pods, [], False, gpu_device, recs)
    try:
        g.ipcache_set([ips[i] for i in sel], [int(ident[i]) for i in sel], [int(meta_id[i]) for i in sel])
        dev = torch.device("cuda", gpu_device)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)  # noqa: E731
        keep = [t(recs.src_ip), t(recs.dst_ip), t(recs.bytes), t(recs.meta), t(recs.ports), t(recs.dns_id)]
        cols = GpuAgg.device_columns(*keep)  # (the tensors must outlive the decode)
        n = len(recs.src_ip)
        out = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(6)]
        g.hubble_decode_device(cols, n, out)
        g.sync()
        got = [o.cpu().numpy().view(np.uint32) for o in out]
    finally:
        g.close()
    ipc = {O.int2ip(ips[i]): H.IPCacheEntry(int(ident[i]), None if meta_id[i] == 0xFFFFFFFF else int(meta_id[i]))
           for i in sel}
    meta = {i: ("p%d" % i, "n%d" % i) for i in range(len(ips))}
    dd = dns_dict(recs)
    kinds = set()
    for i in range(n):
        f = R.flow_from_record(int(recs.src_ip[i]), int(recs.dst_ip[i]), int(recs.bytes[i]), int(recs.meta[i]),
                               int(recs.ports[i]), int(recs.dns_id[i]), dd)
        s = H.decode_endpoint(ipc, meta, f.ip.source)
        d = H.decode_endpoint(ipc, meta, f.ip.destination)
        assert (got[0][i], got[1][i]) == (s.identity, d.identity), i
        want_meta = [ipc[x].meta if x in ipc and ipc[x].meta is not None else 0xFFFFFFFF
                     for x in (f.ip.source, f.ip.destination)]
        assert [int(got[2][i]), int(got[3][i])] == want_meta, i
        code, payload, text = H.summary(f)
        kinds.add(code)
        assert int(got[4][i]) == code, i
        if code == H.SUM_DNS:  # the host renders from the dictionary entry and the DNS type
            e = dd[int(got[5][i]) & 0x3FFFFFFF]
            l7 = {1: "REQUEST", 2: "RESPONSE"}.get(int(got[5][i]) >> 30, "UNKNOWN_L7_TYPE")
            assert H.dns_summary(O.DNS(rcode=e.rcode, query=e.query, qtypes=e.qtypes, ips=e.ips), l7) == text, i
        else:
            assert int(got[5][i]) == payload and H.render_summary(code, int(got[5][i])) == text, i
    assert kinds == {H.SUM_NONE, H.SUM_TCP, H.SUM_UDP, H.SUM_DROP, H.SUM_DNS}
