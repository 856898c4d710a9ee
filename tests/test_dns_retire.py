"""DNS id lifecycle (gpuagg_dns_retire): ids no DNS group-by key
references are retired and reused, so the payload dictionary of an always-on agent does not
grow without bound across epochs.  The series must stay bit-exact against the oracle
(dns.go:102-238 through oracle/oracle.py) before and after ids are reused.  Runs on the CPU
backend here and on gfx950 (`gpu` cases)."""

import numpy as np
import pytest

from retina_amd import _abi
from retina_amd import workloads as W

from .helpers import diff_series, make_engine, oracle_series

SPEC = W.C5_SPEC  # tcpflags + retransmissions + DNS request / response, local context


def _recs(seed):
    pods = W.make_pods(300, seed=41)
    return pods, W.gen_records(20_000, pods, seed=seed, drop_frac=0.0, retrans_frac=0.05, dns_frac=0.5,
                               n_queries=400)


def _intern(g, recs):
    """Interns recs' payloads; returns recs.dns_id mapped to the engine's ids."""
    ids = np.array([g.dns_intern(p.rcode, p.qtypes, p.query, p.ips, p.num_answers) for p in recs.dns],
                   np.uint32)
    out = recs.dns_id.copy()
    is_dns = ((recs.meta >> np.uint32(8)) & np.uint32(0xFF)) == np.uint32(W.V_DNS)
    out[is_dns] = ids[recs.dns_id[is_dns]]
    return ids, out


def _submit(g, recs, dns_id):
    g.submit_numpy(W.Records(recs.src_ip, recs.dst_ip, recs.bytes, recs.meta, recs.ports, dns_id))
    g.sync()


def _check_epochs(flags, device):
    pods, a = _recs(41)
    _, b = _recs(42)
    g = make_engine(pods, SPEC, False, device, flags=flags)
    try:
        ids_a, dns_a = _intern(g, a)
        assert list(ids_a) == list(range(len(a.dns)))
        extra = [g.dns_intern(0, "A", "unused%d.example.com" % k, "", 0) for k in range(3)]
        _submit(g, a, dns_a)
        want_a = oracle_series(a, pods, SPEC, remote=False)
        assert g.snapshot() == want_a
        # only the payloads no key references go (the 3 extra ones, and payloads whose rows
        # had no pod on the side a local-context DNS series is keyed by): the series stay
        assert g.dns_retire() == []  # phase 1: unreferenced ids turn idle
        retired = g.dns_retire()      # phase 2: still unreferenced -> retired
        assert set(extra) <= set(retired) and len(retired) < len(a.dns)
        got = g.snapshot()
        assert got == want_a, diff_series(got, want_a)
        assert g.dns_retire() == []
        # epoch reset: every id is unreferenced, retired, and reused lowest first
        g.reset()
        assert g.dns_retire() == []
        assert sorted(g.dns_retire() + retired) == list(range(len(a.dns) + len(extra)))
        assert g.snapshot() == {}
        ids_b, dns_b = _intern(g, b)
        assert len(set(ids_b.tolist())) == len(b.dns)
        n_old = len(a.dns) + len(extra)
        assert sorted(ids_b.tolist())[: min(n_old, len(b.dns))] == list(range(min(n_old, len(b.dns))))
        _submit(g, b, dns_b)
        want_b = oracle_series(b, pods, SPEC, remote=False)
        got = g.snapshot()
        assert got == want_b, diff_series(got, want_b)
        assert any(k[0].endswith("dns_response_count") for k in want_b)
        # an interned payload is found again under its (reused) id
        p = b.dns[0]
        assert g.dns_intern(p.rcode, p.qtypes, p.query, p.ips, p.num_answers) == ids_b[0]
    finally:
        g.close()


def _check_contexts(flags, device):
    """One dictionary over a node's contexts: an id referenced on any context stays; a
    context with another dictionary is refused; the merge still sees equal dictionaries."""
    from retina_amd import GpuAggError
    pods, a = _recs(43)
    g0 = make_engine(pods, SPEC, False, device, flags=flags)
    g1 = make_engine(pods, SPEC, False, device, flags=flags)
    try:
        _, dns0 = _intern(g0, a)
        _, dns1 = _intern(g1, a)
        half = len(a) // 2
        first = W.Records(*(getattr(a, k)[:half] for k in ("src_ip", "dst_ip", "bytes", "meta", "ports", "dns_id")),
                          a.dns)
        second = W.Records(*(getattr(a, k)[half:] for k in ("src_ip", "dst_ip", "bytes", "meta", "ports",
                                                             "dns_id")), a.dns)
        _submit(g0, first, dns0[:half])
        _submit(g1, second, dns1[half:])
        g0.reset()  # g0's keys are gone; g1 still references its half's ids
        assert g0.dns_retire([g1]) == []
        retired = set(g0.dns_retire([g1]))
        used1 = set(dns1[half:][((second.meta >> np.uint32(8)) & np.uint32(0xFF)) == np.uint32(W.V_DNS)].tolist())
        # every id g1's half does not use is retired (and some of its half's ids too: rows
        # without a pod on the keyed side leave no series)
        assert set(range(len(a.dns))) - used1 <= retired and len(retired) < len(a.dns)
        g0.merge_from([g1])
        want = oracle_series(second, pods, SPEC, remote=False)
        got = g0.snapshot()
        assert got == want, diff_series(got, want)
        g1.dns_intern(0, "A", "only-on-g1.example.com", "", 0)
        with pytest.raises(GpuAggError) as e:
            g0.dns_retire([g1])
        assert e.value.code == _abi.EINVAL
    finally:
        g0.close()
        g1.close()


@pytest.fixture(scope="module")
def lib():
    from retina_amd import build
    build.build()
    return _abi.load()


def test_retire_across_epochs_cpu(lib):
    _check_epochs(_abi.FLAG_CPU_BACKEND, 0)


def test_retire_over_contexts_cpu(lib):
    _check_contexts(_abi.FLAG_CPU_BACKEND, 0)


@pytest.mark.gpu
def test_retire_across_epochs_gpu(gpu_device):
    _check_epochs(0, gpu_device)


@pytest.mark.gpu
def test_retire_over_contexts_gpu(gpu_device):
    _check_contexts(0, gpu_device)


def test_idle_id_handed_out_again_survives(lib):
    """An idle id that the producer interns again before the next call is not retired; a
    late record naming an already retired id is not rendered but counted as lost."""
    pods, a = _recs(44)
    g = make_engine(pods, SPEC, False, 0, flags=_abi.FLAG_CPU_BACKEND)
    try:
        p = a.dns[0]
        i0 = g.dns_intern(p.rcode, p.qtypes, p.query, p.ips, p.num_answers)
        j = g.dns_intern(0, "AAAA", "gone.example.com", "", 0)
        assert g.dns_retire() == []                     # both idle
        assert g.dns_intern(p.rcode, p.qtypes, p.query, p.ips, p.num_answers) == i0  # revived
        assert g.dns_retire() == [j]
        # a DNS request from a pod (egress, as dns_linux.go reports queries) with the live id
        # i0 counts; a late one with the retired id j is not rendered but counted as lost
        is_dns = np.nonzero(((a.meta >> np.uint32(8)) & np.uint32(0xFF)) == np.uint32(W.V_DNS))[0]
        row = next(int(r) for r in is_dns
                   if oracle_series(W.Records(*(getattr(a, k)[r:r + 1] for k in ("src_ip", "dst_ip", "bytes",
                                                                                 "meta", "ports", "dns_id")),
                                              a.dns), pods, SPEC, remote=False))

        def req(dns_id):
            return W.Records(a.src_ip[row:row + 1], a.dst_ip[row:row + 1], a.bytes[row:row + 1],
                             a.meta[row:row + 1], a.ports[row:row + 1], np.array([dns_id], np.uint32))
        _submit(g, req(i0), np.array([i0], np.uint32))
        base = g.snapshot()
        assert any(k[0].split("_")[-2] in ("request", "response") for k in base) and g.last_dropped == 0
        _submit(g, req(j), np.array([j], np.uint32))
        assert g.snapshot() == base
        assert g.last_dropped == 1
    finally:
        g.close()
