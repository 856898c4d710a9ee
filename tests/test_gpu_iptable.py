"""Both HBM images of the IP -> pod map agree with the oracle: the radix table (pod IPs
in few /16 prefixes, the default for cluster CIDRs) and the bucketized cuckoo table
(IPs spread over more than 64 prefixes, or GPUAGG_FLAG_NO_RADIX_IP_TABLE)."""

import numpy as np
import pytest

from retina_amd import workloads as W

from .helpers import diff_series, engine_series, oracle_series

pytestmark = pytest.mark.gpu


def _scattered_pods(n, seed):
    """Pods whose IPs span thousands of /16 prefixes (radix table not applicable)."""
    pods = W.make_pods(n, seed=seed)
    rng = np.random.default_rng(seed)
    remap = {}
    for ip in pods.ips.tolist():
        remap[ip] = int(rng.integers(1, 2**32 - 1))
    eps = [W.Endpoint(e.namespace, e.name, [remap[x] for x in e.ips], e.owner_refs) for e in pods.endpoints]
    ips = np.array([remap[x] for x in pods.ips.tolist()], np.uint32)
    return W.Pods(eps, ips, pods.ip_owner)


@pytest.mark.parametrize("layout", ["radix", "bucket-flag", "bucket-scattered"])
@pytest.mark.parametrize("remote,spec", [(False, W.LOCAL_FWD_DROP + W.C5_SPEC), (True, W.C1_REMOTE)],
                         ids=["local", "remote"])
def test_ip_table_layouts(gpu_device, layout, remote, spec):
    pods = _scattered_pods(3000, 5) if layout == "bucket-scattered" else W.make_pods(3000, seed=5)
    recs = W.gen_records(80_000, pods, seed=6, drop_frac=0.1, retrans_frac=0.05, dns_frac=0.1,
                         udp_frac=0.1, n_queries=300)
    kw = {"flags": 4} if layout == "bucket-flag" else {}
    got = engine_series(recs, pods, spec, remote, gpu_device, host_fed=False, **kw)
    want = oracle_series(recs, pods, spec, remote)
    assert got == want, diff_series(got, want)
    assert len(want) > 100
