"""The CPU backend (GPUAGG_FLAG_CPU_BACKEND, retina_amd/csrc/gpuagg_cpu.cpp): the same
C ABI on host threads for nodes without a gfx950 device.  Runs here (no GPU) against the
oracle with the GPU parity cases, and covers the other entry points the Go plugin uses:
raw perf-record decode, sketches, node-apiserver latency, enriched flows, Hubble decode,
the multi-context merge and slot retirement."""

import zlib

import numpy as np
import pytest

from oracle import decode as DEC
from oracle import records as R
from oracle import sketch as S
from retina_amd import workloads as W

from .helpers import diff_series, engine_series, make_engine, oracle_series
from .test_gpu_parity import CASES, DNS_ALL, MIX, TCP_ALL, spec

CPU = 128  # GPUAGG_FLAG_CPU_BACKEND


@pytest.fixture(scope="module", autouse=True)
def lib():
    from retina_amd import _abi, build
    build.build()
    return _abi.load()


@pytest.mark.parametrize("cid,sp,remote,gen", CASES, ids=[c[0] for c in CASES])
def test_parity_vs_oracle(cid, sp, remote, gen):
    pods = W.make_pods(400, seed=11)
    recs = W.gen_records(30_000, pods, seed=zlib.crc32(cid.encode()) & 0xFFFF, **gen)
    want = oracle_series(recs, pods, sp, remote)
    got = engine_series(recs, pods, sp, remote, host_fed=True, chunks=3, flags=CPU)
    assert got == want, diff_series(got, want)


def test_empty_and_stats():
    from retina_amd import GpuAgg
    pods = W.make_pods(50, seed=1)
    g = make_engine(pods, W.LOCAL_FWD_DROP, False, flags=CPU)
    try:
        assert g.snapshot() == {}
        st = g.stats()
        assert st["records"] == 0
        assert GpuAgg  # the same class drives both backends
    finally:
        g.close()


def test_raw_decode_path():
    """Raw packetparser / dropreason records decoded on the host equal the oracle decode."""
    pods = W.make_pods(300, seed=5)
    sp = spec(["forward_count", "forward_bytes", "drop_count", "drop_bytes", "tcp_flag_gauges"],
              ["namespace", "podname", "port"])
    pk = W.gen_raw_packets(20_000, pods, seed=6, odd_frac=0.05)
    dr = W.gen_raw_drops(10_000, pods, seed=7)
    bp, _ = DEC.decode_packets(pk)
    bd, _ = DEC.decode_drops(dr)
    recs = W.Records(*[np.concatenate([getattr(bp, k), getattr(bd, k)]) for k in
                       ("src_ip", "dst_ip", "bytes", "meta", "ports", "dns_id")])
    want = oracle_series(recs, pods, sp, False)
    from retina_amd import _abi
    g = make_engine(pods, sp, False, flags=CPU)
    try:
        g.submit_raw(_abi.RAW_PACKET, pk)
        g.submit_raw(_abi.RAW_DROP, dr)
        got = g.snapshot()
    finally:
        g.close()
    assert got == want, diff_series(got, want)


def test_sketches_bit_exact():
    pods = W.make_pods(500, seed=8)
    recs = W.gen_records(60_000, pods, seed=9, flows=20_000, n_dst=5_000)
    g = make_engine(pods, W.LOCAL_FWD_DROP, False, flags=CPU, cms_depth=4, cms_width_log2=12, hll_precision=10)
    try:
        g.submit_numpy(recs)
        g.sync()
        cms, hll = g.cms_array(), g.hll_array()
    finally:
        g.close()
    from .test_gpu_sketch import _src_slots
    want = np.zeros((4, 1 << 12), np.uint32)
    S.cms_update(want, recs.src_ip, recs.dst_ip, recs.ports, recs.meta & np.uint32(0xFF))
    assert np.array_equal(cms, want)
    regs = np.zeros_like(hll)
    slot = _src_slots(pods, recs.src_ip)
    ok = (slot >= 0) & (slot < regs.shape[0])
    S.hll_update(regs, slot[ok], recs.dst_ip[ok], 10)
    assert np.array_equal(hll, regs) and hll.any()


def test_latency_matches_oracle():
    from .latency_helpers import as_state, oracle_latency
    api = [W.ip_le(10, 255, 0, 1), W.ip_le(10, 255, 0, 2)]
    sp = [{"metric_name": "node_apiserver_latency"}, {"metric_name": "node_apiserver_handshake_latency"},
          {"metric_name": "node_apiserver_no_response"}]
    pods = W.make_pods(100, seed=11)
    recs = W.gen_latency_records(400, pods, api, seed=12, background=3000)
    want = as_state(oracle_latency(recs, api))
    g = make_engine(pods, sp, False, flags=CPU)
    try:
        g.set_apiserver_ips(api)
        n = len(recs.src_ip)
        hb = g.alloc_batch(n)
        for a, b in ((0, n // 3), (n // 3, n)):  # two batches: requests carried across
            hb.fill(recs, a, b - a)
            g.submit(hb, b - a)
        st = g.latency_state()
    finally:
        g.close()
    assert {k: st[k] for k in want} == want
    assert want["latency_count"] > 0 and want["no_response"] > 0


def test_retire_slots_pod_churn():
    """Pod churn past max_slots on the CPU backend (the retirement must
    zero the dead slots' bins on the host and never reach a device launch): three
    generations of 100 pods in 128 slots; each retirement frees exactly the old
    generation, its series vanish and the slots are reused."""
    from .test_gpu_lifecycle import FWD_DROP, _oracle
    from .helpers import oracle_cache
    g, prev = None, None
    try:
        for gen in range(3):
            pods = W.make_pods(100, seed=50 + gen, apiserver=False)
            pods.endpoints[:] = [W.Endpoint("gen%d" % gen, e.name, e.ips, e.owner_refs) for e in pods.endpoints]
            if g is None:
                g = make_engine(pods, FWD_DROP, False, flags=CPU, max_slots=128, max_ips=512, hll_precision=8)
            else:
                for e in prev.endpoints:
                    g.cache_delete_endpoint(e.namespace, e.name)
                g.cache_commit(version=2 * gen)
                assert g.retire_slots() == 100
                assert g.snapshot() == {}  # every counter of the dead generation cleared
                assert not g.hll_array().any()
                assert g.retire_slots() == 0
                g.load_endpoints(pods.endpoints, version=2 * gen + 1)
            recs = W.gen_records(20_000, pods, seed=60 + gen)
            g.submit_numpy(recs)
            got = g.snapshot()
            want = _oracle(recs, oracle_cache(pods), FWD_DROP)
            assert got == want, diff_series(got, want)
            assert {dict(k[1])["namespace"] for k in got} == {"gen%d" % gen}
            assert g.stats()["records"] == 20_000 * (gen + 1)
            prev = pods
    finally:
        if g is not None:
            g.close()


def test_merge_and_enrich():
    """Two CPU contexts fed the direction-free shards and merged equal one context;
    enriched-flow slots equal the IP cache's pods."""
    from retina_amd import dist as D
    pods = W.make_pods(400, seed=13)
    recs = W.gen_records(40_000, pods, seed=14, **MIX)
    sp = spec(["forward_count", "forward_bytes", "drop_count", "drop_bytes", "dns_request_count"],
              ["ip", "namespace", "podname"], ["podname", "port"])
    want = oracle_series(recs, pods, sp, True)
    parts = [make_engine(pods, sp, True, recs=recs, flags=CPU) for _ in range(2)]
    try:
        for r, g in enumerate(parts):
            g.submit_numpy(D.shard_records(recs, 2, r))
        parts[0].merge_from(parts[1:])
        got = parts[0].snapshot()
        rest = parts[1].snapshot()
        hb = parts[0].alloc_batch(1000)
        hb.fill(recs, 0, 1000)
        s, d = parts[0].submit_enrich(hb, 1000)
    finally:
        for g in parts:
            g.close()
    assert got == want, diff_series(got, want)
    assert rest == {}
    cache = R.build_cache([R.EndpointSpec(e.namespace, e.name, list(e.ips), e.owner_refs) for e in pods.endpoints])
    from oracle import oracle as O
    for i in range(1000):
        obj = cache.get_obj_by_ip(O.int2ip(int(recs.src_ip[i])))
        assert (s[i] >= 0) == isinstance(obj, O.RetinaEndpoint)


@pytest.mark.parametrize("limit,chunks", [(300, 1), (300, 4), (100_000, 1)])
def test_latency_capacity_and_touch(limit, chunks):
    """The ttlcache's capacity (latency.go LIMIT, here also a small gpuagg_config
    latency_limit) and its touch on a Get hit, on the CPU backend against the oracle:
    a burst keeps more requests live than the limit (the least recently touched are
    evicted, uncounted), repeated requests are kept alive by the touch; across batches
    the carried entries keep their LRU order."""
    from .latency_helpers import as_state, oracle_latency
    api = [W.ip_le(10, 255, 0, 1), W.ip_le(10, 255, 0, 2)]
    sp = [{"metric_name": "node_apiserver_latency"}, {"metric_name": "node_apiserver_handshake_latency"},
          {"metric_name": "node_apiserver_no_response"}]
    n_req = 1_200 if limit < 1000 else 130_000
    recs = W.gen_latency_burst(n_req, api, seed=limit + chunks, spacing_ns=100_000 if limit < 1000 else 1_000,
                               background=500)
    m = oracle_latency(recs, api, limit=limit)
    want = as_state(m, capacity=True)
    assert want["capacity_evictions"] > 0 and want["peak_live"] == limit
    pods = W.make_pods(20, seed=3)
    g = make_engine(pods, sp, False, flags=CPU, latency_limit=0 if limit == 100_000 else limit)
    try:
        g.set_apiserver_ips(api)
        n = len(recs.src_ip)
        hb = g.alloc_batch(n)
        bounds = np.linspace(0, n, chunks + 1).astype(int)
        for a, b in zip(bounds[:-1], bounds[1:]):
            hb.fill(recs, int(a), int(b - a))
            g.submit(hb, int(b - a))
        st = g.latency_state()
    finally:
        g.close()
    assert {k: st[k] for k in want} == want
    assert st["limit"] == limit
    # the touch: without it the late replies (650 ms after their first request) find nothing
    assert want["latency_buckets"][10] > 0


def test_exposition_text_cpu_backend():
    """gpuagg_result_render_text on the CPU backend equals the oracle's exposition, with
    values on both sides of Go's 'g' notation switch (1e6: byte sums of jumbo packets,
    trailing zeros, 2^53 and beyond) and a label value that needs escaping; the text is
    rendered once and the sized second call returns the same bytes."""
    import ctypes as C
    from oracle import exposition as X
    from oracle import oracle as O
    pods = W.make_pods(200, seed=91)
    recs = W.gen_records(20_000, pods, seed=92, drop_frac=0.1, retrans_frac=0.05, udp_frac=0.1)
    pods.endpoints[7] = W.Endpoint('ns"q', 'pod\\x\nq', pods.endpoints[7].ips, pods.endpoints[7].owner_refs)
    recs.src_ip[:500] = pods.endpoints[7].ips[0]
    sizes = [1, 999_999, 1_000_000, 1_230_000, 4_000_000_000, 9_007_199_254_740_992 // 4096, 123_456_789]
    for k, b in enumerate(sizes):  # a few big packets: forward_bytes well past 1e6 (and 2^53)
        recs.bytes[1000 + 64 * k:1000 + 64 * k + 64] = min(b, 0xFFFFFFFF)
    sp = spec(["forward_count", "forward_bytes", "drop_count", "drop_bytes"], ["namespace", "podname"])
    g = make_engine(pods, sp, False, flags=CPU)
    try:
        for _ in range(3):
            g.submit_numpy(recs)
        r = C.c_void_p()
        assert g.lib.gpuagg_snapshot(g.h, C.byref(r)) == 0
        try:
            n = C.c_size_t()
            assert g.lib.gpuagg_result_render_text(r, None, 0, C.byref(n)) == 0
            buf = C.create_string_buffer(n.value + 1)
            assert g.lib.gpuagg_result_render_text(r, buf, n.value + 1, C.byref(n)) == 0
            text = buf.value.decode()
            small = C.create_string_buffer(8)
            assert g.lib.gpuagg_result_render_text(r, small, 8, C.byref(n)) != 0  # too small: refused
            ptr, n2 = C.c_void_p(), C.c_size_t()  # the zero-copy form: the same bytes
            assert g.lib.gpuagg_result_text(r, C.byref(ptr), C.byref(n2)) == 0
            assert C.string_at(ptr.value, n2.value) == buf.raw[:n.value] and n2.value == n.value
        finally:
            g.lib.gpuagg_result_free(r)
    finally:
        g.close()
    from .helpers import oracle_cache
    m = O.Module(remote_context=False)
    m.reconcile(R.spec_from_json(sp))
    for _ in range(3):
        R.replay(R.Batch(recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports, recs.dns_id),
                 oracle_cache(pods), m)
    want = X.render(m.series())
    assert text == want
    assert "e+" in text and 'pod\\\\x\\nq' in text


@pytest.mark.parametrize("src,dst", [(["ip", "port"], None),  # few labels: one packed rank key
                                     (["ip", "namespace", "podname", "workload", "service", "port"],
                                      ["ip", "namespace", "podname", "workload", "service", "port"])],
                         ids=["packed-key", "rank-rows"])
def test_exposition_order_large_families(src, dst):
    """Families past the parallel sort's threshold (65536 series) come out in
    client_golang's order -- label values compared in label-name order -- whichever key
    the sort uses: the ranks packed into one 128-bit key, or rank rows when too many
    labels make them wider (oracle.exposition.render over the engine's own series)."""
    from oracle import exposition as X
    pods = W.make_pods(3000, seed=5)
    recs = W.gen_records(400_000, pods, seed=6, flows=300_000, n_dst=50_000)
    sp = spec(["forward_count", "forward_bytes"], src, dst)
    g = make_engine(pods, sp, True, flags=CPU, sparse_capacity_log2=21)
    try:
        g.submit_numpy(recs)
        text = g.snapshot_text()
        series = g.snapshot()
    finally:
        g.close()
    fam = sum(1 for k in series if k[0].endswith("forward_count"))
    assert fam > 65536
    assert text == X.render(series)


@pytest.mark.parametrize("cid,sp,remote,gen", CASES, ids=[c[0] for c in CASES])
def test_exposition_order_every_case(cid, sp, remote, gen):
    """The exposition text of every parity case (all families: directions, drop reasons,
    flags, DNS payloads, workloads, ports and "unknown" values) is the oracle's rendering of
    the same series: the sort tokens order each label exactly as its strings."""
    from oracle import exposition as X
    pods = W.make_pods(200, seed=23)
    recs = W.gen_records(20_000, pods, seed=zlib.crc32(cid.encode()) & 0xFFFF, **gen)
    g = make_engine(pods, sp, remote, recs=recs, flags=CPU)
    try:
        g.submit_numpy(recs)
        text = g.snapshot_text()
        series = g.snapshot()
    finally:
        g.close()
    assert text == X.render(series)


def test_exposition_order_across_growth_and_churn():
    """The cached render tables (canonical slot attributes per slots version, DNS payload
    tokens per table size) follow the engine between snapshots: new DNS payloads interned
    and pods deleted, added and retired in between still render in the oracle's order."""
    from oracle import exposition as X
    pods = W.make_pods(200, seed=31)
    sp = spec(TCP_ALL + DNS_ALL, ["namespace", "podname"])
    a = W.gen_records(20_000, pods, seed=32, **MIX)
    g = make_engine(pods, sp, False, recs=a, flags=CPU)
    try:
        g.submit_numpy(a)
        assert g.snapshot_text() == X.render(g.snapshot())
        more = W.make_pods(260, seed=33)
        for ep in pods.endpoints[:60]:
            g.cache_delete_endpoint(ep.namespace, ep.name)
        for ep in more.endpoints[200:]:
            g.cache_update_endpoint(ep)
        g.cache_commit(1)
        g.retire_slots()
        b = W.gen_records(20_000, more, seed=34, **dict(MIX, n_queries=500))
        ids = np.array([g.dns_intern(p.rcode, p.qtypes, p.query, p.ips, p.num_answers) for p in b.dns],
                       np.uint32)
        assert ids.max() >= len(a.dns)  # the table grew
        has = b.dns_id < len(b.dns)
        b.dns_id[has] = ids[b.dns_id[has]]
        g.submit_numpy(b)
        series = g.snapshot()
        assert any(k[0].endswith("dns_request_count") for k in series)
        assert g.snapshot_text() == X.render(series)
    finally:
        g.close()


def test_scrape_buffers_reused_across_results():
    """The scrape's buffers go back to the context's pool when a result is freed and the
    next snapshot reuses them: results held at the same time, freed in either order and
    re-taken, all render the same text, and a result outliving its context stays valid."""
    import ctypes as C
    from oracle import exposition as X
    pods = W.make_pods(300, seed=41)
    recs = W.gen_records(30_000, pods, seed=42, **MIX)
    sp = spec(["forward_count", "forward_bytes", "drop_count"], ["ip", "podname"], ["namespace", "port"])
    g = make_engine(pods, sp, True, recs=recs, flags=CPU)

    def snap():
        r = C.c_void_p()
        assert g.lib.gpuagg_snapshot(g.h, C.byref(r)) == 0
        return r

    def text(r):
        p, n = C.c_void_p(), C.c_size_t()
        assert g.lib.gpuagg_result_text(r, C.byref(p), C.byref(n)) == 0
        return C.string_at(p.value, n.value)

    try:
        g.submit_numpy(recs)
        want = X.render(g.snapshot()).encode()
        a, b = snap(), snap()  # two alive: the second takes fresh buffers
        assert text(a) == want and text(b) == want
        g.lib.gpuagg_result_free(a)
        c = snap()  # reuses a's buffers
        assert text(c) == want
        g.lib.gpuagg_result_free(c)
        g.lib.gpuagg_result_free(b)
        d = snap()
    finally:
        g.close()
    assert text(d) == want  # the context is gone; the result's buffers are its own
    g.lib.gpuagg_result_free(d)


def test_result_text_concurrent_readers():
    """Two /metrics handlers reading one result: gpuagg_result_text renders once
    (std::call_once) and both readers get the same buffer and length."""
    import ctypes as C
    import threading
    pods = W.make_pods(300, seed=71)
    sp = [{"metric_name": m, "source_labels": ["namespace", "podname"]}
          for m in ("forward_count", "forward_bytes", "drop_count", "drop_bytes")]
    recs = W.gen_records(50_000, pods, seed=72, drop_frac=0.2)
    g = make_engine(pods, sp, False, flags=128)
    try:
        hb = g.alloc_batch(len(recs.src_ip))
        hb.fill(recs)
        g.submit(hb, len(recs.src_ip))
        for _ in range(5):
            r = C.c_void_p()
            assert g.lib.gpuagg_snapshot(g.h, C.byref(r)) == 0
            out = []

            def read():
                p, n = C.c_void_p(), C.c_size_t()
                assert g.lib.gpuagg_result_text(r, C.byref(p), C.byref(n)) == 0
                out.append((p.value, n.value, C.string_at(p, n.value)))
            th = [threading.Thread(target=read) for _ in range(4)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            g.lib.gpuagg_result_free(r)
            assert len(out) == 4 and len({(a, b) for a, b, _ in out}) == 1 and len({t for _, _, t in out}) == 1
            assert out[0][1] > 0
    finally:
        g.close()
