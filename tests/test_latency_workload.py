"""The latency workload exercises every branch of the restated TTL join (CPU)."""

import numpy as np

from retina_amd import workloads as W

from .latency_helpers import as_state, oracle_latency

API = [W.ip_le(10, 255, 0, 1), W.ip_le(10, 255, 0, 2)]


def test_latency_workload_covers_the_join():
    pods = W.make_pods(50, seed=1)
    recs = W.gen_latency_records(300, pods, API, seed=2, background=500)
    m = oracle_latency(recs, API)
    st = as_state(m)
    assert st["latency_count"] > 500 and st["handshake_count"] > 100
    assert st["no_response"] > 10 and m.peak_live < 100_000
    assert min(st["latency_buckets"][i] for i in (0, 2, 4, 6, 8, 10)) > 0  # every integer bucket
    assert not np.all(np.diff(recs.time_ns.astype(np.int64)) >= 0)  # out-of-order rows exist
