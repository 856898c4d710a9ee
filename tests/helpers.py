"""Shared harness: the same seeded records through the oracle and through the engine."""

from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from oracle import oracle as O
from oracle import records as R
from retina_amd import workloads as W


def oracle_cache(pods: W.Pods) -> O.Cache:
    eps = [R.EndpointSpec(e.namespace, e.name, list(e.ips),
                          None if e.owner_refs is None else list(e.owner_refs)) for e in pods.endpoints]
    return R.build_cache(eps)


def dns_dict(recs: W.Records) -> Dict[int, R.DnsEntry]:
    return {i: R.DnsEntry(p.rcode, p.qtypes, p.query, p.ips, p.num_answers) for i, p in enumerate(recs.dns)}


def oracle_series(recs: W.Records, pods: W.Pods, spec: List[dict], remote: bool):
    module = O.Module(remote_context=remote)
    module.reconcile(R.spec_from_json(spec))
    b = R.Batch(recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports, recs.dns_id)
    R.replay(b, oracle_cache(pods), module, dns_dict(recs))
    return module.series()


def make_engine(pods: W.Pods, spec: List[dict], remote: bool, device: int = 0,
                recs: Optional[W.Records] = None, **kw):
    from retina_amd import GpuAgg
    kw.setdefault("max_slots", len(pods.endpoints) + 64)
    kw.setdefault("max_ips", max(16, len(pods.ips)))
    kw.setdefault("sparse_capacity_log2", 20)
    g = GpuAgg(device=device, remote_context=remote, **kw)
    g.reconcile(spec)
    g.load_endpoints(pods.endpoints)
    if recs is not None:
        intern_dns(g, recs)
    return g


def intern_dns(g, recs: W.Records) -> None:
    for i, p in enumerate(recs.dns):
        got = g.dns_intern(p.rcode, p.qtypes, p.query, p.ips, p.num_answers)
        assert got == i, "dns ids must be assigned in first-seen order"


def to_device(recs: W.Records, device: int = 0):
    import torch
    dev = torch.device("cuda", device)

    def t(a):
        return torch.from_numpy(a.view(np.int32)).to(dev)
    return [t(recs.src_ip), t(recs.dst_ip), t(recs.bytes), t(recs.meta), t(recs.ports), t(recs.dns_id)]


def engine_series(recs: W.Records, pods: W.Pods, spec: List[dict], remote: bool, device: int = 0,
                  host_fed: bool = True, chunks: int = 1, **kw):
    from retina_amd import GpuAgg
    g = make_engine(pods, spec, remote, device, recs, **kw)
    try:
        n = len(recs)
        bounds = np.linspace(0, n, chunks + 1).astype(int)
        if host_fed:
            for a, b in zip(bounds[:-1], bounds[1:]):
                part = W.Records(recs.src_ip[a:b], recs.dst_ip[a:b], recs.bytes[a:b], recs.meta[a:b],
                                 recs.ports[a:b], recs.dns_id[a:b])
                g.submit_numpy(part)
        else:
            ts = to_device(recs, device)
            for a, b in zip(bounds[:-1], bounds[1:]):
                cols = GpuAgg.device_columns(*[x[a:] for x in ts])
                g.submit_device(cols, int(b - a))
            g.sync()
        return g.snapshot()
    finally:
        g.close()


def diff_series(a: dict, b: dict, limit: int = 10) -> str:
    keys = set(a) | set(b)
    bad = [(k, a.get(k), b.get(k)) for k in sorted(keys) if a.get(k) != b.get(k)]
    return "%d mismatches of %d/%d series; first: %r" % (len(bad), len(a), len(b), bad[:limit])
