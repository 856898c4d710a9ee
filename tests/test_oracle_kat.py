"""Pins the CPU oracle to the reference's own known-answer tests (tests/golden/reference_kat.json,
transcribed from forward_test.go, drops_test.go, tcpflags_test.go, types_test.go, dns_test.go,
enricher_test.go and utils_linux_test.go)."""

import json
import os

import pytest

from oracle import oracle as O

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kat.json")))


def mk_flow(d):
    if d is None:
        return None
    f = O.Flow(verdict=d["verdict"], traffic_direction=d.get("traffic_direction", 0))
    if d.get("source") is not None:
        f.source = O.Endpoint(d["source"]["namespace"], d["source"]["pod_name"])
    if d.get("destination") is not None:
        f.destination = O.Endpoint(d["destination"]["namespace"], d["destination"]["pod_name"])
    if d.get("ip") is not None:
        f.ip = O.IP(d["ip"]["source"], d["ip"]["destination"], 1)
    if d.get("l4") is not None:
        fl = d["l4"]["flags"]
        f.l4 = O.L4("TCP", 0, 0, None if fl is None else O.TCPFlags(**fl))
    return f


@pytest.mark.parametrize("case", KAT["ctx_options"], ids=lambda c: c["name"])
def test_ctx_options(case):
    c = O.ContextOptions(case["opts"], O.CTX_SOURCE if case["ctx"] == "source" else O.CTX_DESTINATION)
    assert c.get_labels() == case["labels"]
    assert c.get_values(mk_flow(case["flow"])) == case["values"]


@pytest.mark.parametrize("case", KAT["dns_labels"], ids=lambda c: c["name"])
def test_dns_labels(case):
    d = O.DNSMetrics(O.MetricsContextOptions("dns"), O.REMOTE_CONTEXT)
    d.src_ctx = None if case["local_opts"] is None else O.ContextOptions(case["local_opts"], O.CTX_LOCAL)
    got = (O.DNS_REQUEST_LABELS if case["kind"] == "request" else O.DNS_RESPONSE_LABELS) + d._ctx_labels()
    assert got == case["want"]


def dns_flow(qtype, nanswers, ips, tdir=0):
    f = O.Flow(traffic_direction=tdir)
    meta = O.RetinaMetadata()
    O.add_dns_info(f, meta, qtype, 0, "bing.com", ["A"], nanswers, ips)
    return f


@pytest.mark.parametrize("case", KAT["dns_values"], ids=lambda c: c["name"])
def test_dns_values(case):
    d = O.DNSMetrics(O.MetricsContextOptions("dns"), O.REMOTE_CONTEXT)
    d.metric_name = case["metric_name"]
    f = None if case["input"] is None else dns_flow(*case["input"])
    got = d.request_values(f) if case["call"] == "request" else d.response_values(f)
    assert got == case["want"]


class _MockCtx:
    def __init__(self, out):
        self.out = out

    def get_local_ctx_values(self, f):
        return self.out


@pytest.mark.parametrize("case", KAT["dns_local_ctx"], ids=lambda c: c["name"])
def test_dns_local_ctx(case):
    d = O.DNSMetrics(O.MetricsContextOptions("dns_response_count", ["podname"]), O.LOCAL_CONTEXT)
    d.init(O.DNS_RESPONSE_COUNTER)
    d.vec.label_names = O.DNS_RESPONSE_LABELS + ["a", "b"]
    d.src_ctx = _MockCtx(case["local_values"])
    f = None if case["tdir"] is None else dns_flow("R", 1, ["1.1.1.1"], case["tdir"])
    if f is None:
        d.src_ctx.get_local_ctx_values(None)  # processLocalCtxFlow(nil): map nil -> no update
        assert d.vec.calls == 0
        return
    d.process_local_ctx_flow(f)
    if case["want"] is None:
        assert d.vec.calls == 0
    else:
        assert d.vec.calls == 1
        assert list(d.vec.series) == [tuple(case["want"])]


CTORS = {"forward": O.ForwardMetrics, "drop": O.DropCountMetrics, "tcpflags": O.TCPMetrics}
INIT_NAMES = {"forward": ["forward_count", "forward_bytes"], "drop": ["drop_count", "drop_bytes"],
              "tcpflags": ["tcp_flag_gauges"]}


@pytest.mark.parametrize("case", KAT["metric_objects"], ids=lambda c: c["family"] + ":" + c["name"])
def test_metric_objects(case):
    opts = O.MetricsContextOptions(**case["opts"])
    ctx = O.LOCAL_CONTEXT if case["local"] else ""
    for name in INIT_NAMES[case["family"]]:
        m = CTORS[case["family"]].new(opts, ctx)
        if case["nil_obj"]:
            assert m is None
            continue
        assert m is not None
        m.init(name)
        assert m.adv_enable == case["adv"]
        assert m.get_labels() == case["labels"]
        m.process_flow(mk_flow(case["flow"]))
        assert m.vec.calls == case["metric_call"]


def test_enricher_secondary_ips():
    e = KAT["enricher"]
    c = O.Cache()
    for ep in e["endpoints"]:
        c.update_retina_endpoint(O.RetinaEndpoint(
            name=ep["name"], namespace=ep["namespace"], ipv4=ep["ipv4"],
            other_ipv4s=ep["other_ipv4s"], owner_refs=[O.Workload(*w) for w in ep["owner_refs"]]))
    f = O.Flow(ip=O.IP(e["flow"]["source"], e["flow"]["destination"], 1))
    f = O.enrich(c, f)
    assert [f.source.namespace, f.source.pod_name] == e["want_source"]
    assert [f.destination.namespace, f.destination.pod_name] == e["want_destination"]


def test_to_flow():
    t = KAT["to_flow"]
    s, d, sp, dp, proto = t["args"]
    f = O.to_flow(s, d, sp, dp, proto, 1, O.VERDICT_FORWARDED)
    assert [f.ip.source, f.ip.destination, f.ip.ip_version] == t["want_ip"]
    assert [f.l4.source_port, f.l4.destination_port] == t["want_ports"]
    for obs, point in t["obs_points"]:
        assert O.to_flow(s, d, sp, dp, proto, obs, O.VERDICT_FORWARDED).trace_observation_point == point
    f.extensions.bytes = t["packet_size"]
    assert O.packet_size(f) == t["packet_size"]


@pytest.mark.parametrize("reason,name", KAT["drop_reason"])
def test_drop_reason(reason, name):
    f = O.drop_flow("1.1.1.1", "2.2.2.2", 1, 2, 6, reason, 10)
    assert f.verdict == O.VERDICT_DROPPED
    assert O.drop_reason_description(f) == name


def test_decode_packet_roundtrip():
    """struct packet (conntrack.c:34-49) decode: LE IPs, byte-swapped ports, flags."""
    raw = O.PACKET_STRUCT.pack(5, 1400, O.ip2int("10.0.0.1"), O.ip2int("10.0.0.2"),
                               O.host_to_net_short(443), O.host_to_net_short(8080), 1, 2, 3, 4,
                               1, 2, 6, O.TCP_FLAG_SYN | O.TCP_FLAG_ACK, True, 0, 0, 0, 0)
    f = O.decode_packet(raw)
    assert (f.ip.source, f.ip.destination) == ("10.0.0.1", "10.0.0.2")
    assert (f.l4.source_port, f.l4.destination_port) == (443, 8080)
    assert f.traffic_direction == 2 and f.is_reply is True
    assert O.tcp_flag_values(f.l4.flags) == ["SYNACK"]
    assert f.extensions.bytes == 1400 and f.extensions.tcp_id == 0  # obs 1: no TCP id


def test_enum_names_unknown_numbers():
    assert O.enum_string(O.DROP_REASON_NAMES, 7) == "7"
    assert O.traffic_direction_string(3) == "3"


def _obj_kind(obj):
    if obj is None:
        return None
    if isinstance(obj, O.RetinaEndpoint):
        return {"kind": "pod", "namespace": obj.namespace, "name": obj.name}
    if isinstance(obj, O.RetinaSvc):
        return {"kind": "svc", "namespace": obj.namespace, "name": obj.name}
    return {"kind": "node", "namespace": "", "name": obj.name}


def run_cache_ops(c, ops):
    """Applies a cache_sequences op list to the oracle Cache; yields (op, error, got)."""
    for op in ops:
        kind = op["op"]
        err, got = False, None
        try:
            if kind == "update_endpoint":
                ips = op["ips"]
                c.update_retina_endpoint(O.RetinaEndpoint(name=op["name"], namespace=op["namespace"],
                                                          ipv4=ips[0] if ips else None, other_ipv4s=ips[1:]))
            elif kind == "update_service":
                c.update_retina_svc(O.RetinaSvc(op["name"], op["namespace"], op["ip"]))
            elif kind == "update_node":
                c.update_retina_node(O.RetinaNode(op["name"], op["ip"]))
            elif kind == "delete_endpoint":
                c.delete_retina_endpoint(op["namespace"] + "/" + op["name"])
            elif kind == "delete_service":
                c.delete_retina_svc(op["namespace"] + "/" + op["name"])
            elif kind == "delete_node":
                c.delete_retina_node(op["name"])
            elif kind == "get":
                got = _obj_kind(c.get_obj_by_ip(op["ip"]))
        except (ValueError, KeyError):
            err = True
        yield op, err, got


@pytest.mark.parametrize("case", KAT["cache_sequences"], ids=lambda c: c["name"])
def test_cache_sequences(case):
    """pkg/controllers/cache/cache_test.go: last writer wins across pods, services and
    nodes; deleting a missing pod is ignored, a missing service or node is an error."""
    for op, err, got in run_cache_ops(O.Cache(), case["ops"]):
        if op["op"] == "get":
            assert got == op["want"], (case["src"], op)
        else:
            assert err == op["error"], (case["src"], op)


@pytest.mark.parametrize("case", KAT["reconcile"], ids=lambda c: c["name"])
def test_reconcile_transitions(case):
    """metrics_module_test.go TestModule_Reconcile: the registry is rebuilt unless the spec
    equals the current one; invalid metric names register no vector."""
    from oracle import records as R
    m = O.Module(remote_context=True)  # the test's Module has no daemonConfig: remote context
    if case["prior"]:
        m.reconcile(R.spec_from_json(case["prior"]))
    if case["current_spec"] is not None:
        m.current_spec = R.spec_from_json(case["current_spec"])
    before = dict(m.registry)
    rebuilt = m.reconcile_spec(R.spec_from_json(case["spec"]))
    assert rebuilt == (not case["expect_no_calls"])
    if case["expect_no_calls"]:
        assert m.registry == before
    else:
        assert set(m.registry) == {o["metric_name"] for o in case["spec"]}
        vecs = {n: m.registry[n].vec for n in m.registry}
        for n, v in vecs.items():  # Init creates a vector only for the exact *_count / *_bytes names
            assert (v is not None) == (n in ("drop_count", "drop_bytes", "forward_count", "forward_bytes")), n


def test_exposition_layout_pinned_by_reference_sample():
    """The text layout of oracle/exposition.py (which the engine's gpuagg_result_render_text
    equals byte for byte, test_cpu_backend.py) against the scrape the reference's docs print
    (docs/06-Troubleshooting/basic-metrics.md:86-124): family order, HELP / TYPE lines,
    label-pair and metric order, Go FormatFloat('g', -1) values (1.9064666952e+10, 34713)."""
    from oracle import exposition as X
    ex = KAT["exposition_sample"]
    fams = {k: (t, h) for k, (t, h) in ex["families"].items()}
    series = {(m, tuple(lab.items())): v for m, lab, v in ex["series"]}
    assert X.render(series, fams) == "".join(line + "\n" for line in ex["text"])


def test_traffic_direction_names_from_reference_identifiers():
    """The direction label values (TrafficDirection.String(), forward.go:116) are the proto
    value names that the reference's Go identifiers carry (flow_utils.go:75-91):
    protoc-gen-go names each constant <Enum>_<value name>."""
    names = {i.split("_", 1)[1] for i in KAT["traffic_direction_identifiers"]["identifiers"]}
    assert names == set(O.TRAFFIC_DIRECTION_NAMES.values())
