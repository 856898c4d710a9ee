"""Host-side lifecycle of the engine on the GPU, each against the reference's rules:

* the native IP cache follows cache.go's update/delete semantics (whole-object deletion
  on an IP collision, services and nodes owning IPs, stale IPs of an updated pod);
* dense counters / HLL rows grow with the slots in use and keep their values;
* slots the IP table no longer references retire and are reused (pod churn past
  max_slots), their series cleared;
* reconcile with equal context options is a no-op (metrics_module.go:142-166);
* the single-process multi-context merge (gpuagg_merge) equals one engine;
* the Prometheus text exposition equals the oracle's rendering;
* a full group-by table no longer fails the snapshot: the loss is reported with it.
"""

import numpy as np
import pytest

from oracle import exposition as X
from oracle import oracle as O
from oracle import records as R
from retina_amd import workloads as W

from .helpers import diff_series, make_engine, oracle_cache, to_device

pytestmark = pytest.mark.gpu

FWD_DROP = W.LOCAL_FWD_DROP


def _ep(e: W.Endpoint) -> O.RetinaEndpoint:
    return O.RetinaEndpoint(name=e.name, namespace=e.namespace, ipv4=O.int2ip(e.ips[0]),
                            other_ipv4s=[O.int2ip(x) for x in e.ips[1:]],
                            owner_refs=None if e.owner_refs is None else [O.Workload(k, n) for k, n in e.owner_refs])


def _oracle(recs, cache, spec, remote=False):
    m = O.Module(remote_context=remote)
    m.reconcile(R.spec_from_json(spec))
    R.replay(R.Batch(recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports, recs.dns_id), cache, m)
    return m.series()


def _submit(g, recs, device):
    from retina_amd import GpuAgg
    g.submit_device(GpuAgg.device_columns(*to_device(recs, device)), len(recs))
    g.sync()


def test_cache_semantics_match_reference(gpu_device):
    from retina_amd import _abi
    from retina_amd.engine import GpuAggError
    pods = W.make_pods(300, seed=31, secondary_frac=0.5)
    eps = pods.endpoints
    new1, new2 = W.ip_le(10, 200, 0, 1), W.ip_le(10, 200, 0, 2)
    ops = [  # (engine op, oracle op)
        # a new pod takes pod 10's first IP: pod 10 is deleted with ALL its IPs
        ("ep", W.Endpoint("ns-x", "pod-x", [eps[10].ips[0], new1], [("Deployment", "dx")])),
        # a service takes pod 20's IP, a node pod 30's: both pods deleted
        ("svc", ("ns-s", "svc-s", int(eps[20].ips[0]))),
        ("node", ("node-n", int(eps[30].ips[0]))),
        # pod 40 updated to a new IP list: its old IPs keep pointing at it (stale)
        ("ep", W.Endpoint(eps[40].namespace, eps[40].name, [new2], eps[40].owner_refs)),
        # pod 50 deleted; pod 60 re-owned (another identity, another slot)
        ("del", (eps[50].namespace, eps[50].name)),
        ("ep", W.Endpoint(eps[60].namespace, eps[60].name, list(eps[60].ips), [("StatefulSet", "ss")])),
        # a pod takes the service's IP back; the service is gone
        ("ep", W.Endpoint("ns-y", "pod-y", [int(eps[20].ips[0])], None)),
    ]
    cache = oracle_cache(pods)
    g = make_engine(pods, FWD_DROP, False, gpu_device)
    try:
        for kind, arg in ops:
            if kind == "ep":
                g.cache_update_endpoint(arg)
                cache.update_retina_endpoint(_ep(arg))
            elif kind == "svc":
                g.cache_update_service(*arg)
                cache.update_retina_svc(O.RetinaSvc(arg[1], arg[0], O.int2ip(arg[2])))
            elif kind == "node":
                g.cache_update_node(*arg)
                cache.update_retina_node(O.RetinaNode(arg[0], O.int2ip(arg[1])))
            elif kind == "del":
                g.cache_delete_endpoint(*arg)
                cache.delete_retina_endpoint(arg[0] + "/" + arg[1])
        with pytest.raises(GpuAggError) as ei:  # deleteSvc of an unknown key is an error
            g.cache_delete_service("ns-s", "svc-s")  # (deleted when pod-y took its IP)
        assert ei.value.code == _abi.ENOTFOUND
        g.cache_commit(version=7)
        # records between every IP of interest
        special = np.array([x for e in eps[:70] for x in e.ips] + [new1, new2], np.uint32)
        recs = W.gen_records(60_000, pods, seed=32, pod_frac=1.0)
        rng = np.random.default_rng(33)
        recs.src_ip[:] = special[rng.integers(0, len(special), len(recs))]
        recs.dst_ip[::2] = special[rng.integers(0, len(special), (len(recs) + 1) // 2)]
        _submit(g, recs, gpu_device)
        got = g.snapshot()
    finally:
        g.close()
    want = _oracle(recs, cache, FWD_DROP)
    assert got == want, diff_series(got, want)
    # the ops did what the reference does: pod 10 lost every IP, pod 40 kept its stale one
    assert all(cache.get_obj_by_ip(O.int2ip(ip)) is None for ip in eps[10].ips[1:])
    assert cache.get_obj_by_ip(O.int2ip(eps[40].ips[0])).name == eps[40].name


def test_slots_grow_and_keep_counters(gpu_device):
    """Dense counters and HLL rows are sized by the slots in use: 100 pods, then 5000 more
    (a relayout), counters accumulated before and after the growth are all kept."""
    pods = W.make_pods(5_100, seed=41)
    few = W.Pods(pods.endpoints[:100], pods.ips, pods.ip_owner)
    recs = W.gen_records(200_000, pods, seed=42)
    half = len(recs) // 2
    a = W.Records(*(x[:half] for x in (recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports, recs.dns_id)))
    b = W.Records(*(x[half:] for x in (recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports, recs.dns_id)))
    g = make_engine(few, FWD_DROP, False, gpu_device, max_slots=8192, max_ips=16384, hll_precision=8)
    try:
        s0 = g.state()
        _submit(g, a, gpu_device)
        g.load_endpoints(pods.endpoints[100:], version=2)
        s1 = g.state()
        _submit(g, b, gpu_device)
        got = g.snapshot()
        hll = g.hll_array()
    finally:
        g.close()
    assert s1.dense_len > s0.dense_len and s1.hll_len > s0.hll_len
    cache = oracle_cache(few)
    want = _oracle(a, cache, FWD_DROP)
    for e in pods.endpoints[100:]:
        cache.update_retina_endpoint(_ep(e))
    for k, v in _oracle(b, cache, FWD_DROP).items():
        want[k] = want.get(k, 0) + v
    assert got == want, diff_series(got, want)
    assert hll.shape[0] >= 5_100


def test_pod_churn_past_max_slots(gpu_device):
    """max_slots=128: three generations of 100 pods each.  At each epoch boundary the old
    generation is deleted from the cache, the table re-committed and its slots retired
    (their counters cleared); the engine never runs out of slots and each epoch's
    snapshot holds exactly the current generation's series."""
    g, prev = None, None
    try:
        for gen in range(3):
            pods = W.make_pods(100, seed=50 + gen, apiserver=False)
            pods.endpoints[:] = [W.Endpoint("gen%d" % gen, e.name, e.ips, e.owner_refs) for e in pods.endpoints]
            if g is None:
                g = make_engine(pods, FWD_DROP, False, gpu_device, max_slots=128, max_ips=512)
            else:
                for e in prev.endpoints:
                    g.cache_delete_endpoint(e.namespace, e.name)
                g.cache_commit(version=2 * gen)
                assert g.retire_slots() == 100
                g.load_endpoints(pods.endpoints, version=2 * gen + 1)
            recs = W.gen_records(50_000, pods, seed=60 + gen)
            _submit(g, recs, gpu_device)
            got = g.snapshot()
            want = _oracle(recs, oracle_cache(pods), FWD_DROP)
            assert got == want, diff_series(got, want)
            assert {dict(k[1])["namespace"] for k in got} == {"gen%d" % gen}
            prev = pods
    finally:
        if g is not None:
            g.close()


def test_reconcile_same_options_keeps_counters(gpu_device):
    pods = W.make_pods(200, seed=71)
    recs = W.gen_records(30_000, pods, seed=72)
    g = make_engine(pods, FWD_DROP, False, gpu_device)
    try:
        _submit(g, recs, gpu_device)
        before = g.snapshot()
        # the same options, labels reordered and entries permuted: MetricsContextOptionsCompare
        # calls them equal, Module.Reconcile does nothing
        g.reconcile([{"metric_name": m["metric_name"], "source_labels": list(reversed(m["source_labels"]))}
                     for m in reversed(FWD_DROP)])
        assert g.snapshot() == before and before
        # a real change re-creates the metrics (empty state)
        g.reconcile(FWD_DROP[:2])
        assert g.snapshot() == {}
    finally:
        g.close()


def test_merge_contexts_equals_single(gpu_device):
    from retina_amd import dist as D
    pods = W.make_pods(800, seed=81)
    recs = W.gen_records(400_000, pods, seed=82, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.1,
                         udp_frac=0.1, n_queries=500)
    sketch = dict(cms_depth=4, cms_width_log2=14, hll_precision=9)
    out = []
    for remote, spec, kw in ((False, FWD_DROP + W.C5_SPEC, sketch), (True, W.C1_REMOTE, {})):
        one = make_engine(pods, spec, remote, gpu_device, recs, **kw)
        _submit(one, recs, gpu_device)
        want = one.snapshot()
        wc = one.cms_array() if kw else None
        wh = one.hll_array() if kw else None
        one.close()
        parts = [make_engine(pods, spec, remote, gpu_device, recs, **kw) for _ in range(3)]
        for r, g in enumerate(parts):
            _submit(g, D.shard_records(recs, 3, r), gpu_device)
        parts[0].merge_from(parts[1:])
        got = parts[0].snapshot()
        rest = [p.snapshot() for p in parts[1:]]
        gc = parts[0].cms_array() if kw else None
        gh = parts[0].hll_array() if kw else None
        for p in parts:
            p.close()
        assert got == want, diff_series(got, want)
        assert rest == [{}, {}]
        if kw:
            assert np.array_equal(gc, wc) and np.array_equal(gh, wh)
        out.append(len(got))
    assert min(out) > 100


def test_merge_rccl_one_device(gpu_device):
    """gpuagg_merge over in-process RCCL (contexts on distinct devices): on a one-GPU lease
    the communicator has one rank -- ncclCommInitAll, the in-place reduces of every state
    array and the entry transfer run, and the state is unchanged (a second merge reuses the
    communicator).  Multi-device RCCL merges are unmeasured here; the peer-copy path (same
    device) is test_merge_contexts_equals_single."""
    pods = W.make_pods(500, seed=83)
    recs = W.gen_records(200_000, pods, seed=84, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.1,
                         udp_frac=0.1, n_queries=300)
    sketch = dict(cms_depth=4, cms_width_log2=14, hll_precision=9)
    for remote, spec, kw in ((False, FWD_DROP + W.C5_SPEC, sketch), (True, W.C1_REMOTE, {})):
        g = make_engine(pods, spec, remote, gpu_device, recs, **kw)
        try:
            _submit(g, recs, gpu_device)
            want = g.snapshot()
            wc = g.cms_array() if kw else None
            g.merge_from([])  # one context: a one-rank communicator
            g.merge_from([])
            got = g.snapshot()
            if kw:
                assert np.array_equal(g.cms_array(), wc)
        finally:
            g.close()
        assert got == want and len(got) > 100, diff_series(got, want)


@pytest.mark.parametrize("remote,spec", [(False, FWD_DROP + W.C5_SPEC), (True, W.C1_REMOTE)],
                         ids=["local", "remote"])
def test_exposition_text_matches_oracle(gpu_device, remote, spec):
    pods = W.make_pods(300, seed=91)
    recs = W.gen_records(20_000, pods, seed=92, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.1,
                         udp_frac=0.1, n_queries=200)
    # a pod name that needs escaping in a label value
    pods.endpoints[7] = W.Endpoint('ns"q', 'pod\\x\nq', pods.endpoints[7].ips, pods.endpoints[7].owner_refs)
    recs.src_ip[:500] = pods.endpoints[7].ips[0]
    g = make_engine(pods, spec, remote, gpu_device, recs)
    try:
        _submit(g, recs, gpu_device)
        text = g.snapshot_text()
        fams = g.snapshot_families()
    finally:
        g.close()
    cache = oracle_cache(pods)
    m = O.Module(remote_context=remote)
    m.reconcile(R.spec_from_json(spec))
    from .helpers import dns_dict
    R.replay(R.Batch(recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports, recs.dns_id), cache, m,
             dns_dict(recs))
    want = X.render(m.series())
    assert text == want
    assert fams and all(fams[k] == X.FAMILIES[k] for k in fams)
    assert 'pod\\\\x\\nq' in text


def test_full_table_reports_loss(gpu_device):
    """A 16-slot group-by table overflows: the snapshot still returns (the dense series
    stay exact) and reports the lost updates (gpuagg_result_dropped)."""
    pods = W.make_pods(100, seed=95)
    recs = W.gen_records(20_000, pods, seed=96)
    g = make_engine(pods, W.C1_REMOTE, True, gpu_device, sparse_capacity_log2=4)
    try:
        _submit(g, recs, gpu_device)
        got = g.snapshot()
        assert g.last_dropped > 0 and len(got) > 0
    finally:
        g.close()
