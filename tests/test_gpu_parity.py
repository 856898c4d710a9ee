"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle, bit-exact.

Every case generates seeded records, replays them through oracle.Module one flow at a
time, runs the same records through libgpuagg.so on the MI355X, and compares every
Prometheus series (metric, label tuple) -> exact integer value.
"""

import zlib

import numpy as np
import pytest

from retina_amd import workloads as W

from .helpers import diff_series, engine_series, oracle_series

pytestmark = pytest.mark.gpu

ALL6 = ["ip", "namespace", "podname", "workload", "service", "port"]


def spec(names, src=None, dst=None):
    return [{"metric_name": n, "source_labels": src, "destination_labels": dst} for n in names]


FWD_DROP = ["forward_count", "forward_bytes", "drop_count", "drop_bytes"]
TCP_ALL = ["tcp_flag_gauges", "tcp_retransmission_count"]
DNS_ALL = ["dns_request_count", "dns_response_count"]
EVERYTHING = FWD_DROP + TCP_ALL + DNS_ALL

MIX = dict(drop_frac=0.1, retrans_frac=0.05, dns_frac=0.2, udp_frac=0.15, other_proto_frac=0.05,
           n_queries=300)

CASES = [
    # (id, spec, remote, gen kwargs)
    ("local-dense-ns-pod", spec(FWD_DROP, ["namespace", "podname"]), False, {}),
    ("local-dense-workload", spec(FWD_DROP + TCP_ALL, ["workload"]), False, MIX),
    ("local-dense-service-only", spec(FWD_DROP, ["service"]), False, {}),
    ("local-c1-ip-ns-pod-wl", spec(FWD_DROP, W.C1_LABELS), False, {}),
    ("local-all6", spec(EVERYTHING, ALL6), False, MIX),
    ("local-no-labels", spec(FWD_DROP, []), False, {}),
    ("remote-c1", spec(FWD_DROP, W.C1_LABELS, W.C1_LABELS), True, {}),
    ("remote-plain", spec(FWD_DROP + TCP_ALL + DNS_ALL), True, MIX),
    ("remote-dst-only", spec(EVERYTHING, None, ["namespace", "podname", "port"]), True, MIX),
    ("remote-all6-both", spec(EVERYTHING, ALL6, ALL6), True, MIX),
    ("c5-local", W.C5_SPEC, False, dict(drop_frac=0.0, retrans_frac=0.05, dns_frac=0.35, n_queries=500)),
    ("odd-rows-local", spec(EVERYTHING, ["namespace", "podname", "port"]), False, dict(MIX, odd_frac=0.2)),
    ("odd-rows-remote", spec(EVERYTHING, ["ip", "podname"], ["workload", "port"]), True, dict(MIX, odd_frac=0.2)),
]


@pytest.mark.parametrize("cid,sp,remote,gen", CASES, ids=[c[0] for c in CASES])
def test_parity_vs_oracle(gpu_device, cid, sp, remote, gen):
    pods = W.make_pods(400, seed=11)
    recs = W.gen_records(30_000, pods, seed=zlib.crc32(cid.encode()) & 0xFFFF, **gen)
    want = oracle_series(recs, pods, sp, remote)
    got = engine_series(recs, pods, sp, remote, gpu_device, host_fed=True, chunks=3)
    assert got == want, diff_series(got, want)
    if cid in ("local-all6", "remote-all6-both"):
        got_dev = engine_series(recs, pods, sp, remote, gpu_device, host_fed=False, chunks=2)
        assert got_dev == want, diff_series(got_dev, want)


def test_zipf_contention(gpu_device):
    """C4 shape: heavy-hitter source pods hammer the same counters (atomic contention)."""
    pods = W.make_pods(300, seed=4)
    recs = W.gen_records(60_000, pods, seed=4, zipf=1.2)
    sp = spec(FWD_DROP, ["namespace", "podname"])
    want = oracle_series(recs, pods, sp, False)
    got = engine_series(recs, pods, sp, False, gpu_device, host_fed=False)
    assert got == want, diff_series(got, want)


def test_empty_and_single(gpu_device):
    pods = W.make_pods(50, seed=1)
    sp = spec(FWD_DROP, ["namespace", "podname"])
    recs = W.gen_records(1, pods, seed=1, pod_frac=1.0)
    empty = W.Records(*(a[:0] for a in (recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports,
                                         recs.dns_id)))
    assert engine_series(empty, pods, sp, False, gpu_device) == {}
    assert engine_series(recs, pods, sp, False, gpu_device) == oracle_series(recs, pods, sp, False)


def test_sparse_duplicates_merge_and_import(gpu_device):
    """Export/import of the sparse table (the multi-GPU merge path) preserves series."""
    import torch
    from .helpers import make_engine, to_device
    from retina_amd import GpuAgg
    pods = W.make_pods(200, seed=7)
    recs = W.gen_records(20_000, pods, seed=7, **MIX)
    sp = spec(EVERYTHING, ["ip", "namespace", "port"], ["podname"])
    want = oracle_series(recs, pods, sp, True)
    half = len(recs) // 2
    engines = [make_engine(pods, sp, True, gpu_device, recs) for _ in range(2)]
    ts = to_device(recs, gpu_device)
    engines[0].submit_device(GpuAgg.device_columns(*ts), half)
    engines[1].submit_device(GpuAgg.device_columns(*[t[half:] for t in ts]), len(recs) - half)
    for e in engines:
        e.sync()
    buf = torch.empty((1 << 20) * 5, dtype=torch.int64, device="cuda")
    n = engines[1].sparse_export(buf.data_ptr(), 1 << 20)
    engines[0].sparse_import(buf.data_ptr(), n)
    got = engines[0].snapshot()
    for e in engines:
        e.close()
    assert got == want, diff_series(got, want)


def test_endpoint_swap_between_batches(gpu_device):
    """A versioned IP table swap applies to later batches only (cache.go:204-233)."""
    from .helpers import oracle_cache
    from oracle import oracle as O, records as R
    pods = W.make_pods(100, seed=3)
    recs = W.gen_records(10_000, pods, seed=3, pod_frac=1.0)
    sp = spec(FWD_DROP, ["namespace", "podname"])
    # move pod-5's IPs to a new pod identity between the two halves
    moved = W.Endpoint("ns-new", "pod-moved", list(pods.endpoints[5].ips), [("Job", "j")])
    half = len(recs) // 2
    module = O.Module(False)
    module.reconcile(R.spec_from_json(sp))
    cache = oracle_cache(pods)
    b = R.Batch(recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports, recs.dns_id)
    R.replay(b.slice(0, half), cache, module)
    cache.update_retina_endpoint(O.RetinaEndpoint(name="pod-moved", namespace="ns-new",
                                                  ipv4=O.int2ip(moved.ips[0]),
                                                  other_ipv4s=[O.int2ip(x) for x in moved.ips[1:]],
                                                  owner_refs=[O.Workload("Job", "j")]))
    R.replay(b.slice(half, len(recs)), cache, module)
    want = module.series()

    from .helpers import make_engine
    g = make_engine(pods, sp, False, gpu_device)
    first = W.Records(*(a[:half] for a in (recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports, recs.dns_id)))
    second = W.Records(*(a[half:] for a in (recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports, recs.dns_id)))
    g.submit_numpy(first)
    eps = [e for i, e in enumerate(pods.endpoints) if i != 5] + [moved]
    g.load_endpoints(eps, version=2)
    g.submit_numpy(second)
    got = g.snapshot()
    g.close()
    assert got == want, diff_series(got, want)


def test_sketches_bit_exact(gpu_device):
    """Count-min counters and HLL registers equal the numpy restatement bit for bit."""
    from oracle import sketch as S
    from .helpers import make_engine, to_device
    from retina_amd import GpuAgg
    pods = W.make_pods(64, seed=9)
    recs = W.gen_records(200_000, pods, seed=9, udp_frac=0.3)
    sp = spec(["forward_count"], ["namespace"])
    g = make_engine(pods, sp, False, gpu_device, cms_depth=4, cms_width_log2=12, hll_precision=10)
    g.submit_device(GpuAgg.device_columns(*to_device(recs, gpu_device)), len(recs))
    g.sync()
    cms = g.cms_array()
    hll = g.hll_array()
    # restatement
    want_cms = np.zeros((4, 1 << 12), np.uint32)
    S.cms_update(want_cms, recs.src_ip, recs.dst_ip, recs.ports, recs.meta & np.uint32(0xFF))
    assert np.array_equal(cms, want_cms)
    ip_slot = {}
    for s, ep in enumerate(pods.endpoints):
        for ip in ep.ips:
            ip_slot[int(ip)] = s
    slot = np.array([ip_slot.get(int(x), -1) for x in recs.src_ip], np.int64)
    want_hll = np.zeros((64, 1 << 10), np.uint8)
    S.hll_update(want_hll, slot, recs.dst_ip, 10)
    assert np.array_equal(hll[:64], want_hll)
    g.sketch_refresh()
    for s in (1, 5, 9):
        assert abs(g.hll_estimate(s) - S.hll_estimate(want_hll[s])) < 1e-6
    est = g.cms_estimate(int(recs.src_ip[0]), int(recs.dst_ip[0]), int(recs.ports[0]), int(recs.meta[0] & 0xFF))
    assert est >= 1
    g.close()


TIER0 = [c for c in CASES if c[0] in ("local-dense-ns-pod", "local-dense-workload", "odd-rows-local")]


@pytest.mark.parametrize("cid,sp,remote,gen", TIER0, ids=[c[0] for c in TIER0])
def test_parity_without_lds_ip_table(gpu_device, cid, sp, remote, gen):
    """The dense kernel with the IP table in HBM (FLAG_NO_LDS_IP_TABLE) stays exact."""
    from retina_amd import _abi
    pods = W.make_pods(400, seed=11)
    recs = W.gen_records(30_000, pods, seed=zlib.crc32(cid.encode()) & 0xFFFF, **gen)
    want = oracle_series(recs, pods, sp, remote)
    got = engine_series(recs, pods, sp, remote, gpu_device, host_fed=True, chunks=3,
                        flags=_abi.FLAG_NO_LDS_IP_TABLE)
    assert got == want, diff_series(got, want)
