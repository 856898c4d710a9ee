"""Enriched-flow emission (standard mode) on the GPU against the oracle's Enricher.enrich
(enricher.go:102-140), record by record: the endpoint put into flow.Source /
flow.Destination, through the C ABI (gpuagg_enrich_device)."""

import numpy as np
import pytest

from oracle import oracle as O
from oracle import records as R
from retina_amd import workloads as W

from .helpers import dns_dict, make_engine, oracle_cache

pytestmark = pytest.mark.gpu


def _run(g, recs, dev):
    import torch
    from retina_amd import GpuAgg
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)  # noqa: E731
    keep = [t(recs.src_ip), t(recs.dst_ip), t(recs.bytes), t(recs.meta), t(recs.ports), t(recs.dns_id)]
    cols = GpuAgg.device_columns(*keep)  # (the tensors must outlive the launch)
    n = len(recs.src_ip)
    out = [torch.full((n,), -7, dtype=torch.int32, device=dev) for _ in range(2)]
    g.enrich_device(cols, n, out[0], out[1])
    g.sync()
    return [o.cpu().numpy() for o in out]


def _want(cache, recs, slot_of):
    dd = dns_dict(recs)
    ws, wd = [], []
    for i in range(len(recs.src_ip)):
        f = R.flow_from_record(int(recs.src_ip[i]), int(recs.dst_ip[i]), int(recs.bytes[i]), int(recs.meta[i]),
                               int(recs.ports[i]), int(recs.dns_id[i]), dd)
        f = O.enrich(cache, f)
        assert f is not None  # IPv4 u32 records are never dropped by enrich
        for ep, acc in ((f.source, ws), (f.destination, wd)):
            acc.append(-1 if ep is None else slot_of[(ep.namespace, ep.pod_name)])
    return np.array(ws, np.int32), np.array(wd, np.int32)


@pytest.mark.parametrize("n", [40_000, 40_001])  # vector path + a ragged tail
def test_enrich_matches_oracle(gpu_device, n):
    import torch
    pods = W.make_pods(1500, seed=71)
    recs = W.gen_records(n, pods, seed=72, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.1, udp_frac=0.1,
                         n_queries=100)
    g = make_engine(pods, [], False, gpu_device, recs)
    try:
        # a service and a node own pod-range IPs: GetObjByIP finds them, getEndpoint -> nil
        svc_ip, node_ip = int(pods.ips[5]), int(pods.ips[7])
        g.cache_update_service("ns-svc", "svc-a", svc_ip)
        g.cache_update_node("node-a", node_ip)
        g.cache_commit(1)
        slot_of = {}
        for ep in pods.endpoints:
            own = ep.owner_refs[0] if ep.owner_refs else (None, None)
            slot_of[(ep.namespace, ep.name)] = g.slot_intern(ep.namespace, ep.name, own[0], own[1])
        got = _run(g, recs, torch.device("cuda", gpu_device))
    finally:
        g.close()
    cache = oracle_cache(pods)
    cache.update_retina_svc(O.RetinaSvc("svc-a", "ns-svc", O.int2ip(svc_ip)))
    cache.update_retina_node(O.RetinaNode("node-a", O.int2ip(node_ip)))
    ws, wd = _want(cache, recs, slot_of)
    assert (ws == -1).any() and (ws >= 0).any() and (wd >= 0).any()
    np.testing.assert_array_equal(got[0], ws)
    np.testing.assert_array_equal(got[1], wd)


def test_enrich_follows_cache_updates(gpu_device):
    """An updated pod that takes another pod's IP deletes that whole pod (cache.go:204-233,
    394-420); emission after the commit follows the new map, the old one before it."""
    import torch
    pods = W.make_pods(300, seed=73)
    recs = W.gen_records(8_000, pods, seed=74)
    dev = torch.device("cuda", gpu_device)
    g = make_engine(pods, [], False, gpu_device, recs)
    try:
        before = _run(g, recs, dev)
        victim = pods.endpoints[10]
        thief = pods.endpoints[11]
        g.cache_update_endpoint(W.Endpoint(thief.namespace, thief.name, list(thief.ips) + [victim.ips[0]],
                                           thief.owner_refs))
        staged = _run(g, recs, dev)  # not committed yet: the old map
        g.cache_commit(2)
        after = _run(g, recs, dev)
        own = thief.owner_refs[0] if thief.owner_refs else (None, None)
        thief_slot = g.slot_intern(thief.namespace, thief.name, own[0], own[1])
    finally:
        g.close()
    np.testing.assert_array_equal(staged[0], before[0])
    hit = recs.src_ip == victim.ips[0]
    assert hit.any()
    assert (after[0][hit] == thief_slot).all()
    others = ~np.isin(recs.src_ip, np.asarray(victim.ips, np.uint32))
    np.testing.assert_array_equal(after[0][others], before[0][others])


def test_enrich_requires_endpoints(gpu_device):
    import torch
    from retina_amd import GpuAgg
    from retina_amd.engine import GpuAggError
    g = GpuAgg(device=gpu_device, max_slots=64, max_ips=64)
    try:
        g.reconcile([])
        dev = torch.device("cuda", gpu_device)
        z = torch.zeros(64, dtype=torch.int32, device=dev)
        cols = GpuAgg.device_columns(z, z, z, z, z, z)
        with pytest.raises(GpuAggError):
            g.enrich_device(cols, 64, z, z)
    finally:
        g.close()


def test_submit_enrich_host_fed(gpu_device):
    """gpuagg_submit_enrich: the host-fed batch is aggregated (series equal the oracle's)
    and its endpoints come back equal to the device-side emission."""
    import torch
    from .helpers import oracle_series
    pods = W.make_pods(800, seed=75)
    recs = W.gen_records(30_001, pods, seed=76, drop_frac=0.1)
    spec = W.LOCAL_FWD_DROP
    g = make_engine(pods, spec, False, gpu_device, recs)
    try:
        n = len(recs.src_ip)
        hb = g.alloc_batch(n)
        for name in ("src_ip", "dst_ip", "bytes", "meta", "ports", "dns_id"):
            getattr(hb, name)[:n] = getattr(recs, name)
        s_host, d_host = g.submit_enrich(hb, n)
        g.sync()
        got = g.snapshot()
        dev = _run(g, recs, torch.device("cuda", gpu_device))
    finally:
        g.close()
    np.testing.assert_array_equal(s_host, dev[0])
    np.testing.assert_array_equal(d_host, dev[1])
    assert got == oracle_series(recs, pods, spec, remote=False)
