"""Reconcile semantics through the C ABI on the GPU: metric-name resolution, nil vs empty
label slices, reference panics turned into errors (metrics_module.go:205-264,
basemetricsobject.go:31-49, dns.go:352-372)."""

import pytest

from retina_amd import GpuAggError, workloads as W
from retina_amd import _abi

from .helpers import diff_series, engine_series, make_engine, oracle_series

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def data():
    pods = W.make_pods(200, seed=21)
    recs = W.gen_records(20_000, pods, seed=21, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.1,
                         udp_frac=0.1, n_queries=50)
    return pods, recs


NAME_CASES = [
    # names that register but never update, substring dispatch order, case handling
    ([{"metric_name": "forward", "source_labels": ["podname"]}], False),
    ([{"metric_name": "FORWARD_count", "source_labels": ["podname"]}], False),
    ([{"metric_name": "drop_forward", "source_labels": ["podname"]}], False),
    ([{"metric_name": "tcpflag", "source_labels": ["podname"]}], False),
    ([{"metric_name": "tcp_retrans_and_flags", "source_labels": ["podname"]}], False),
    ([{"metric_name": "tcp_nothing", "source_labels": ["podname"]}], False),
    ([{"metric_name": "node_apiserver_latency", "source_labels": ["podname"]}], False),
    ([{"metric_name": "pktmon_something", "source_labels": ["podname"]}], False),
    ([{"metric_name": "forward_count", "source_labels": ["PodName", "NAMESPACE", "bogus"]}], False),
    ([{"metric_name": "forward_count", "source_labels": []}], True),
    ([{"metric_name": "forward_count", "source_labels": [], "destination_labels": []}], True),
    ([{"metric_name": "forward_count", "source_labels": [], "destination_labels": ["podname"]}], True),
    ([{"metric_name": "drop_count", "destination_labels": ["ip"]}], True),
    ([{"metric_name": "forward_count", "source_labels": ["podname"]},
      {"metric_name": "forward_count", "source_labels": ["namespace"]}], False),  # last wins
]


@pytest.mark.parametrize("spec,remote", NAME_CASES, ids=[str(i) for i in range(len(NAME_CASES))])
def test_name_resolution_matches_oracle(gpu_device, data, spec, remote):
    pods, recs = data
    want = oracle_series(recs, pods, spec, remote)
    got = engine_series(recs, pods, spec, remote, gpu_device)
    assert got == want, diff_series(got, want)


def test_reference_panics_are_errors(gpu_device, data):
    pods, _ = data
    g = make_engine(pods, [], False, gpu_device)
    with pytest.raises(GpuAggError) as e:
        g.reconcile([{"metric_name": "forward_count"}])  # local ctx, nil sourceLabels
    assert e.value.code == _abi.EINVAL
    with pytest.raises(GpuAggError) as e:
        g.reconcile([{"metric_name": "dns_lookups", "source_labels": ["podname"]}])
    assert e.value.code == _abi.EINVAL
    with pytest.raises(GpuAggError) as e:
        g.reconcile([{"metric_name": "tcp_flag_a", "source_labels": ["podname"]},
                     {"metric_name": "tcp_flag_b", "source_labels": ["podname"]}])
    assert e.value.code == _abi.EDUPLICATE
    g.close()


def test_reconcile_resets_counters(gpu_device, data):
    pods, recs = data
    sp = W.LOCAL_FWD_DROP
    g = make_engine(pods, sp, False, gpu_device, recs)
    g.submit_numpy(recs)
    assert g.snapshot()
    g.reconcile(sp)  # equal options: Module.Reconcile does nothing (metrics_module.go:142-166)
    assert g.snapshot()
    g.reconcile(sp[:2])  # a change re-creates the metrics ...
    g.reconcile(sp)      # ... and so does changing back
    assert g.snapshot() == {}
    g.submit_numpy(recs)
    assert g.snapshot() == oracle_series(recs, pods, sp, False)
    g.reset()
    assert g.snapshot() == {}
    g.close()
