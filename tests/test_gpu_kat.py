"""The reference's own test sequences through the native engine (tests/golden/reference_kat.json):

* cache_test.go (cache_sequences): the native IP cache (gpuagg_cache_*) applies the same
  update / delete sequences; after each lookup point the installed IP -> pod map, read
  back through gpuagg_enrich_device, names the pod GetObjByIP returns (a service, a node
  or nothing resolve to no endpoint, enricher.go:147-164), and the calls fail where the
  reference returns an error.
* metrics_module_test.go TestModule_Reconcile (reconcile): gpuagg_reconcile rebuilds the
  metric registry -- state reset, then series equal to the oracle's -- except when the
  options equal the current ones, where the accumulated series are kept."""

import json
import os

import numpy as np
import pytest

from retina_amd import workloads as W

from .helpers import diff_series, oracle_series, to_device

pytestmark = pytest.mark.gpu

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kat.json")))


def _ip(s):
    a, b, c, d = (int(x) for x in s.split("."))
    return W.ip_le(a, b, c, d)


@pytest.mark.parametrize("case", KAT["cache_sequences"], ids=lambda c: c["name"])
def test_native_cache_sequences(gpu_device, case):
    import torch
    from retina_amd import GpuAgg, GpuAggError, _abi
    from retina_amd.engine import Endpoint
    g = GpuAgg(device=gpu_device, max_slots=64, max_ips=64, sparse_capacity_log2=10)
    dev = torch.device("cuda", gpu_device)
    try:
        g.reconcile(W.LOCAL_FWD_DROP)
        version = 0
        for op in case["ops"]:
            kind = op["op"]
            if kind == "get":
                version += 1
                g.cache_commit(version)
                ip = torch.tensor([_ip(op["ip"])], dtype=torch.int64).to(torch.int32).to(dev)
                z = torch.zeros(1, dtype=torch.int32, device=dev)
                src = torch.empty(1, dtype=torch.int32, device=dev)
                dst = torch.empty(1, dtype=torch.int32, device=dev)
                g.enrich_device(GpuAgg.device_columns(ip, ip, z, z), 1, src, dst)
                g.sync()
                got = int(src.item())
                w = op["want"]
                want = g.slot_intern(w["namespace"], w["name"]) if w and w["kind"] == "pod" else -1
                assert got == want, (case["src"], op)
                continue
            if kind == "update_service" and op["ip"] is None:
                continue  # a service without an IP is not representable in the C ABI (the Go
                #           caller gets GetPrimaryIP's error before calling)
            try:
                if kind == "update_endpoint":
                    g.cache_update_endpoint(Endpoint(op["namespace"], op["name"], [_ip(x) for x in op["ips"]]))
                elif kind == "update_service":
                    g.cache_update_service(op["namespace"], op["name"], _ip(op["ip"]))
                elif kind == "update_node":
                    g.cache_update_node(op["name"], _ip(op["ip"]))
                elif kind == "delete_endpoint":
                    g.cache_delete_endpoint(op["namespace"], op["name"])
                elif kind == "delete_service":
                    g.cache_delete_service(op["namespace"], op["name"])
                elif kind == "delete_node":
                    g.cache_delete_node(op["name"])
                err = None
            except GpuAggError as e:
                err = e.code
            if op["error"]:
                assert err in (_abi.EINVAL, _abi.ENOTFOUND), (case["src"], op, err)
            else:
                assert err is None, (case["src"], op, err)
    finally:
        g.close()


@pytest.mark.parametrize("case", KAT["reconcile"], ids=lambda c: c["name"])
def test_native_reconcile_transitions(gpu_device, case):
    from retina_amd import GpuAgg
    pods = W.make_pods(300, seed=14)
    recs = W.gen_records(50_000, pods, seed=15)
    g = GpuAgg(device=gpu_device, remote_context=True, max_slots=400, max_ips=800, sparse_capacity_log2=20)
    cols = GpuAgg.device_columns(*to_device(recs, gpu_device))
    try:
        if case["prior"]:
            g.reconcile(case["prior"])
        g.load_endpoints(pods.endpoints)
        if case["prior"]:
            g.submit_device(cols, len(recs))
        before = g.snapshot()
        g.reconcile(case["spec"])  # never an error (the reference returns nil in every case)
        after = g.snapshot()
        if case["expect_no_calls"]:
            assert after == before and len(before) > 0  # spec equals the current one: untouched
            return
        assert after == {}  # registry rebuilt: Clean + ResetAdvancedMetricsRegistry
        g.submit_device(cols, len(recs))
        got = g.snapshot()
    finally:
        g.close()
    want = oracle_series(recs, pods, case["spec"], remote=True)
    assert got == want, diff_series(got, want)
    assert {k[0] for k in got} <= {"networkobservability_adv_" + n for n in
                                   ("drop_count", "drop_bytes", "forward_count", "forward_bytes")}
