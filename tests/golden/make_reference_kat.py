"""Writes reference_kat.json: the known-answer cases of the reference's own Go tests,
transcribed as data (inputs + expected outputs), each citing the test it comes from.

The reference cannot run here (no Go toolchain), so these vectors pin
the oracle.  Run:  python tests/golden/make_reference_kat.py
"""

import json
import os

ALL = ["ip", "namespace", "podName", "Workload", "PORT", "serVICE"]
SRC_ALL = ["source_ip", "source_namespace", "source_podname", "source_workload_kind",
           "source_workload_name", "source_service", "source_port"]
DST_ALL = [s.replace("source_", "destination_") for s in SRC_ALL]
LOC_ALL = [s.replace("source_", "") for s in SRC_ALL]
EMPTY_EP = {"namespace": "", "pod_name": ""}
ALL_FLAGS = {"SYN": True, "FIN": True, "RST": True, "PSH": True, "URG": True, "ECE": True,
             "CWR": True, "ACK": True}


def fl(verdict=0, source=None, destination=None, ip=None, l4=None, tdir=0):
    return {"verdict": verdict, "source": source, "destination": destination, "ip": ip, "l4": l4,
            "traffic_direction": tdir}


def tcp(flags):
    return {"proto": "TCP", "flags": flags}


F, D = 1, 2

kat = {
    # pkg/module/metrics/types_test.go:21-141 (TestNewCtxOps)
    "ctx_options": [
        {"name": "empty opts", "opts": [], "ctx": "source", "labels": [], "flow": fl(),
         "values": []},
        {"name": "source opts 1", "opts": ALL, "ctx": "source", "labels": SRC_ALL, "flow": fl(),
         "values": ["unknown"] * 7},
        {"name": "dest opts 1", "opts": ALL, "ctx": "destination", "labels": DST_ALL, "flow": fl(),
         "values": ["unknown"] * 7},
        {"name": "source opts with flow", "opts": ALL, "ctx": "source", "labels": SRC_ALL,
         "flow": fl(source={"namespace": "ns", "pod_name": "test"}),
         "values": ["unknown", "ns", "test", "unknown", "unknown", "unknown", "unknown"]},
        {"name": "source opts with flow (destination)", "opts": ALL, "ctx": "destination",
         "labels": DST_ALL, "flow": fl(destination={"namespace": "ns", "pod_name": "test"}),
         "values": ["unknown", "ns", "test", "unknown", "unknown", "unknown", "unknown"]},
        {"name": "source opts of ip", "opts": ["ip", "namespace", "podName"], "ctx": "source",
         "labels": ["source_ip", "source_namespace", "source_podname"],
         "flow": fl(source={"namespace": "ns", "pod_name": "test"},
                    ip={"source": "10.0.0.1", "destination": ""}),
         "values": ["10.0.0.1", "ns", "test"]},
        {"name": "dest opts of ip", "opts": ["ip", "namespace", "podName"], "ctx": "destination",
         "labels": ["destination_ip", "destination_namespace", "destination_podname"],
         "flow": fl(destination={"namespace": "ns", "pod_name": "test"},
                    ip={"source": "", "destination": "10.0.0.1"}),
         "values": ["10.0.0.1", "ns", "test"]},
        {"name": "dest opts of ip with no destination info", "opts": ["ip", "namespace", "podName"],
         "ctx": "destination",
         "labels": ["destination_ip", "destination_namespace", "destination_podname"],
         "flow": fl(source={"namespace": "ns", "pod_name": "test"},
                    ip={"source": "10.0.0.1", "destination": ""}),
         "values": ["", "unknown", "unknown"]},
    ],
    # pkg/module/metrics/dns_test.go:24-93 (TestGetLabels)
    "dns_labels": [
        {"name": "basic context request labels", "local_opts": None, "kind": "request",
         "want": ["query_type", "query"]},
        {"name": "basic context response labels", "local_opts": None, "kind": "response",
         "want": ["return_code", "query_type", "query", "response", "num_response"]},
        {"name": "local context request labels",
         "local_opts": ["ip", "namespace", "podname", "service", "port", "workload"],
         "kind": "request",
         "want": ["query_type", "query", "ip", "namespace", "podname", "workload_kind",
                  "workload_name", "service", "port"]},
    ],
    # pkg/module/metrics/dns_test.go:95-194 (TestValues); flows built with AddDNSInfo
    # (qtype, rcode 0, "bing.com", ["A"], num_answers, ips)
    "dns_values": [
        {"name": "basic context", "metric_name": "", "input": None, "call": "response", "want": None},
        {"name": "Query", "metric_name": "dns_request_count", "input": ["Q", 0, []],
         "call": "request", "want": ["A", "bing.com"]},
        {"name": "Response", "metric_name": "dns_response_count", "input": ["R", 1, ["1.1.1.1"]],
         "call": "response", "want": ["NOERROR", "A", "bing.com", "1.1.1.1", "1"]},
        {"name": "UnknownType/DNSRequest", "metric_name": "dns_request_count",
         "input": ["U", 0, []], "call": "response", "want": None},
        {"name": "UnknownType/DNSResponse", "metric_name": "dns_response_count",
         "input": ["U", 0, []], "call": "response", "want": None},
        {"name": "Query/ResponseMetric", "metric_name": "dns_response_count", "input": ["Q", 0, []],
         "call": "request", "want": None},
        {"name": "Response/RequestMetric", "metric_name": "dns_request_count",
         "input": ["R", 1, ["1.1.1.1"]], "call": "response", "want": None},
    ],
    # pkg/module/metrics/dns_test.go:196-315 (TestProcessLocalCtx): getLocalCtxValues mocked
    "dns_local_ctx": [
        {"name": "No context labels", "tdir": None, "local_values": None, "want": None},
        {"name": "Only ingress labels", "tdir": 0,
         "local_values": {"ingress": ["PodA", "NamespaceA"], "egress": None},
         "want": ["NOERROR", "A", "bing.com", "1.1.1.1", "1", "PodA", "NamespaceA"]},
        {"name": "Only egress labels", "tdir": 0,
         "local_values": {"ingress": None, "egress": ["PodA", "NamespaceA"]},
         "want": ["NOERROR", "A", "bing.com", "1.1.1.1", "1", "PodA", "NamespaceA"]},
        {"name": "Both ingress and egress labels with ingress flow", "tdir": 1,
         "local_values": {"ingress": ["PodA", "NamespaceA"], "egress": ["PodB", "NamespaceB"]},
         "want": ["NOERROR", "A", "bing.com", "1.1.1.1", "1", "PodA", "NamespaceA"]},
        {"name": "Both ingress and egress labels with egress flow", "tdir": 2,
         "local_values": {"ingress": ["PodA", "NamespaceA"], "egress": ["PodB", "NamespaceB"]},
         "want": ["NOERROR", "A", "bing.com", "1.1.1.1", "1", "PodB", "NamespaceB"]},
    ],
    # forward_test.go:31-310, drops_test.go:20-299, tcpflags_test.go:20-497:
    # constructor nil-ness, advEnable, label schema and the WithLabelValues call count.
    "metric_objects": [],
    # pkg/enricher/enricher_test.go:41-157: secondary IPs resolve to their pods.
    "enricher": {
        "endpoints": [
            {"name": "pod1", "namespace": "ns1", "ipv4": "1.1.1.1", "other_ipv4s": ["1.1.1.2"],
             "owner_refs": [["Pod", "pod1-deployment"]]},
            {"name": "pod2", "namespace": "ns2", "ipv4": "2.2.2.2", "other_ipv4s": ["2.2.2.3"],
             "owner_refs": [["Pod", "pod2-deployment"]]},
        ],
        "flow": {"source": "1.1.1.2", "destination": "2.2.2.3"},
        "want_source": ["ns1", "pod1"], "want_destination": ["ns2", "pod2"],
    },
    # pkg/utils/utils_linux_test.go:19-73 (TestToFlow) and :75-96 (TestAddPacketSize)
    "to_flow": {
        "args": ["1.1.1.1", "2.2.2.2", 443, 80, 6],
        "want_ip": ["1.1.1.1", "2.2.2.2", 1], "want_ports": [443, 80],
        "obs_points": [[0, "TO_STACK"], [1, "TO_ENDPOINT"], [2, "FROM_NETWORK"],
                       [3, "TO_NETWORK"], [4, "UNKNOWN_POINT"]],
        "packet_size": 100,
    },
    # pkg/utils/utils_linux_test.go:120-167 (TestAddDropReason): verdict DROPPED + reason names
    "drop_reason": [[0, "IPTABLE_RULE_DROP"], [1, "IPTABLE_NAT_DROP"], [5, "CONNTRACK_ADD_DROP"],
                    [6, "UNKNOWN_DROP"]],
}


def mo(family, name, opts, flow, labels, calls, nil=False, adv=False, local=False, src="forward_test.go"):
    kat["metric_objects"].append({"family": family, "name": name, "opts": opts, "flow": flow,
                                  "labels": labels, "metric_call": calls, "nil_obj": nil,
                                  "adv": adv, "local": local, "source": src})


def o(name="", src=None, dst=None):
    return {"metric_name": name, "source_labels": src, "destination_labels": dst}


# forward_test.go:35-278
mo("forward", "empty opts", o(), fl(), ["direction"], 0, nil=True)
mo("forward", "plain opts", o("forward"), fl(F), ["direction"], 1)
mo("forward", "plain opts with nil flow", o("forward"), None, ["direction"], 0)
mo("forward", "plain opts dropped verdict", o("forward"), fl(D), ["direction"], 0)
mo("forward", "source opts 1 without metric name", o(src=ALL), fl(), ["direction"], 0, nil=True)
mo("forward", "source opts 1", o("forward", src=ALL), fl(F), ["direction"] + SRC_ALL, 1, adv=True)
mo("forward", "dest opts 1", o("FORWARD", dst=ALL), fl(F), ["direction"] + DST_ALL, 1, adv=True)
mo("forward", "source opts with flow", o("forward", src=ALL), fl(F, source=EMPTY_EP),
   ["direction"] + SRC_ALL, 1, adv=True)
mo("forward", "drop source opts expect nil", o("drop", src=ALL), fl(F, source=EMPTY_EP),
   ["direction"] + SRC_ALL, 1, nil=True, adv=True)
mo("forward", "source opts with flow dropped verdict", o("forward", src=ALL),
   fl(D, source=EMPTY_EP), ["direction"] + SRC_ALL, 0, adv=True)
mo("forward", "source opts with flow in local context", o("forward", src=ALL),
   fl(F, source=EMPTY_EP), ["direction"] + LOC_ALL, 1, adv=True, local=True)
mo("forward", "dest opts 1 with flow in local context", o("FORWARD", src=ALL),
   fl(F, destination=EMPTY_EP), ["direction"] + LOC_ALL, 1, adv=True, local=True)
mo("forward", "src and dest opts 1 with flow in local context", o("FORWARD", src=ALL),
   fl(F, source=EMPTY_EP, destination=EMPTY_EP), ["direction"] + LOC_ALL, 2, adv=True, local=True)
# drops_test.go:23-265
S = "drops_test.go"
mo("drop", "empty opts", o(), fl(F), ["reason"], 0, nil=True, src=S)
mo("drop", "empty opts dropped", o(), fl(D), ["reason"], 0, nil=True, src=S)
mo("drop", "plain opts", o("drop"), fl(), ["reason", "direction"], 0, src=S)
mo("drop", "plain opts dropped verdict", o("drop"), fl(D), ["reason", "direction"], 1, src=S)
mo("drop", "plain opts dropped verdict nil flow", o("drop"), None, ["reason", "direction"], 0, src=S)
mo("drop", "source opts 1 without metric name", o(src=ALL), fl(D), ["reason", "direction"], 1,
   nil=True, src=S)
mo("drop", "source opts 1", o("drop", src=ALL), fl(D), ["reason", "direction"] + SRC_ALL, 1,
   adv=True, src=S)
mo("drop", "dest opts 1", o("DROP", dst=ALL), fl(D), ["reason", "direction"] + DST_ALL, 1,
   adv=True, src=S)
mo("drop", "source opts with flow", o("drop", src=ALL), fl(D, source=EMPTY_EP),
   ["reason", "direction"] + SRC_ALL, 1, adv=True, src=S)
mo("drop", "forward source opts with flow", o("forward", src=ALL), fl(D, source=EMPTY_EP),
   ["reason", "direction"] + SRC_ALL, 1, nil=True, adv=True, src=S)
mo("drop", "drop source opts with flow in localcontext", o("drop", src=ALL),
   fl(D, source=EMPTY_EP), ["reason", "direction"] + LOC_ALL, 1, adv=True, local=True, src=S)
mo("drop", "drop source opts with destination flow in localcontext", o("drop", src=ALL),
   fl(D, destination=EMPTY_EP), ["reason", "direction"] + LOC_ALL, 1, adv=True, local=True, src=S)
mo("drop", "drop source opts with source and destination flow in localcontext", o("drop", src=ALL),
   fl(D, source=EMPTY_EP, destination=EMPTY_EP), ["reason", "direction"] + LOC_ALL, 2, adv=True,
   local=True, src=S)
# tcpflags_test.go:24-467
S = "tcpflags_test.go"
EXCEPT_ACK = {k: v for k, v in ALL_FLAGS.items() if k != "ACK"}
EXCEPT_SYN = {k: v for k, v in ALL_FLAGS.items() if k != "SYN"}
mo("tcpflags", "empty opts", o(), fl(), [], 1, nil=True, src=S)
mo("tcpflags", "empty opts nil flow", o("tcpflags"), None, ["flag"], 0, src=S)
mo("tcpflags", "plain opts", o("tcpflags"), fl(), ["flag"], 0, src=S)
mo("tcpflags", "source opts 1 without metric name", o(src=ALL), fl(F), ["flag"] + SRC_ALL, 0,
   nil=True, adv=False, src=S)
mo("tcpflags", "source opts 1", o("flag", src=ALL), fl(), ["flag"] + SRC_ALL, 0, adv=True, src=S)
mo("tcpflags", "dest opts 1", o("flag", dst=ALL), fl(F), ["flag"] + DST_ALL, 0, adv=True, src=S)
mo("tcpflags", "source opts with flow", o("flag", src=ALL), fl(F, source=EMPTY_EP),
   ["flag"] + SRC_ALL, 0, adv=True, src=S)
mo("tcpflags", "source opts with flow with flags", o("flag", src=ALL),
   fl(F, source=EMPTY_EP, l4=tcp({"SYN": True})), ["flag"] + SRC_ALL, 1, adv=True, src=S)
mo("tcpflags", "source opts with nil flow", o("flag", src=ALL),
   fl(F, source=EMPTY_EP, l4=tcp(None)), ["flag"] + SRC_ALL, 0, adv=True, src=S)
mo("tcpflags", "source opts with flow with all flags except ack", o("flag", src=ALL),
   fl(F, source=EMPTY_EP, l4=tcp(EXCEPT_ACK)), ["flag"] + SRC_ALL, 7, adv=True, src=S)
mo("tcpflags", "dest opts with flow with all flags", o("flag", dst=ALL),
   fl(F, source=EMPTY_EP, l4=tcp(ALL_FLAGS)), ["flag"] + DST_ALL, 7, adv=True, src=S)
mo("tcpflags", "dest opts with flow with all but syn flags", o("flag", dst=ALL),
   fl(F, source=EMPTY_EP, l4=tcp(EXCEPT_SYN)), ["flag"] + DST_ALL, 7, adv=True, src=S)
mo("tcpflags", "dest opts with flow with all flags dropped verdict", o("flag", dst=ALL),
   fl(D, source=EMPTY_EP, l4=tcp(ALL_FLAGS)), ["flag"] + DST_ALL, 0, adv=True, src=S)
mo("tcpflags", "local ctx dest opts with flow with all flags", o("flag", src=ALL),
   fl(F, source=EMPTY_EP, l4=tcp(ALL_FLAGS)), ["flag"] + LOC_ALL, 7, adv=True, local=True, src=S)
mo("tcpflags", "local ctx no endpoints with all flags", o("flag", src=ALL),
   fl(F, l4=tcp(ALL_FLAGS)), ["flag"] + LOC_ALL, 0, adv=True, local=True, src=S)
mo("tcpflags", "local ctx src and dest opts with flow with all flags", o("flag", src=ALL),
   fl(F, source=EMPTY_EP, destination=EMPTY_EP, l4=tcp(ALL_FLAGS)), ["flag"] + LOC_ALL, 14,
   adv=True, local=True, src=S)

# ---- pkg/controllers/cache/cache_test.go: the IP cache's update / delete / lookup rules ----
def upd_ep(ns, name, ips, error=False):
    return {"op": "update_endpoint", "namespace": ns, "name": name, "ips": ips, "error": error}


def upd_svc(ns, name, ip, error=False):
    return {"op": "update_service", "namespace": ns, "name": name, "ip": ip, "error": error}


def upd_node(name, ip, error=False):
    return {"op": "update_node", "name": name, "ip": ip, "error": error}


def get(ip, kind=None, ns="", name=""):
    return {"op": "get", "ip": ip, "want": None if kind is None else {"kind": kind, "namespace": ns, "name": name}}


kat["cache_sequences"] = [
    {"name": "TestCacheEndpoints", "src": "cache_test.go:31-96", "ops": [
        upd_ep("ns1", "pod1", [], error=True),              # no IPs: ep.IPs() error
        upd_ep("ns1", "pod1", ["1.2.3.4", "1.2.3.5"]),      # IPv4 + OtherIPv4s
        get("1.2.3.4", "pod", "ns1", "pod1"),
        get("1.2.3.5", "pod", "ns1", "pod1"),               # by secondary IP
        {"op": "delete_endpoint", "namespace": "ns1", "name": "pod1", "error": False}]},
    {"name": "TestCacheServices", "src": "cache_test.go:98-140", "ops": [
        upd_svc("ns1", "svc1", None, error=True),           # GetPrimaryIP error
        upd_svc("ns1", "svc1", "1.2.3.4"),
        get("1.2.3.4", "svc", "ns1", "svc1"),
        {"op": "delete_service", "namespace": "ns1", "name": "svc1", "error": False}]},
    {"name": "TestCacheNodes", "src": "cache_test.go:142-173", "ops": [
        upd_node("node1", "1.2.3.4"),
        get("1.2.3.4", "node", "", "node1"),
        {"op": "delete_node", "name": "node1", "error": False}]},
    {"name": "TestAddPodSvcNodeSameIP", "src": "cache_test.go:175-225", "ops": [
        upd_ep("ns1", "pod1", ["1.2.3.4"]),
        upd_svc("ns1", "svc1", "1.2.3.4"),
        get("1.2.3.4", "svc", "ns1", "svc1"),               # the service took the IP
        upd_node("node1", "1.2.3.4"),
        get("1.2.3.4", "node", "", "node1")]},              # then the node
    {"name": "TestAddPodSvcNodeSameIPDiffNS", "src": "cache_test.go:227-278", "ops": [
        upd_ep("ns1", "pod1", ["1.2.3.4"]),
        upd_svc("ns2", "svc1", "1.2.3.4"),
        get("1.2.3.4", "svc", "ns2", "svc1"),
        upd_node("node1", "1.2.3.4"),
        get("1.2.3.4", "node", "", "node1")]},
    {"name": "TestAddPodDiffNs", "src": "cache_test.go:280-322", "ops": [
        upd_ep("ns1", "pod1", ["1.2.3.4"]),
        upd_ep("ns2", "pod1", ["1.2.3.4"]),
        get("1.2.3.4", "pod", "ns2", "pod1")]},             # last writer wins
    {"name": "TestFailDelete", "src": "cache_test.go:324-349", "ops": [
        {"op": "delete_endpoint", "namespace": "ns1", "name": "pod1", "error": False},  # ignored
        {"op": "delete_service", "namespace": "ns1", "name": "svc1", "error": True},
        {"op": "delete_node", "name": "node1", "error": True}]},
]

# ---- pkg/module/metrics/metrics_module_test.go:369-615 (TestModule_Reconcile) ----
# `prior`: the options the module's registry was built from (the test's pre-Init'ed metric
# objects, remote context: the test's Module has no daemonConfig); `current_spec`: the
# module's currentSpec (nil except in the no-op case).  The reference's Reconcile returns
# nil in every case (its updateMetricsContexts logs invalid names instead of failing, so
# the test's expectErr is permissive: `err != nil && !expectErr`); expect_no_calls: the
# spec equals currentSpec, so nothing is re-registered and the registry is left alone.
# AdditionalLabels is not read on the metrics path and is omitted.
def mco(name, src=None, dst=None):
    d = {"metric_name": name}
    if src is not None:
        d["source_labels"] = src
    if dst is not None:
        d["destination_labels"] = dst
    return d


_DC = mco("drop_count", ["ip"], ["pod"])
_FC = mco("forward_count", ["ip"], ["pod"])
kat["reconcile"] = [
    {"name": "Registry is empty and no error", "src": "metrics_module_test.go:427-446",
     "prior": [], "current_spec": None, "spec": [mco("drop_count", ["ip", "pod"], ["pod"])],
     "reference_error": False, "expect_no_calls": False},
    {"name": "Registry is not empty and no error", "src": "metrics_module_test.go:447-475",
     "prior": [_DC, _FC], "current_spec": None,
     "spec": [mco("drop_count", ["ip", "pod"], ["pod"]), mco("forward_count", ["ip", "pod"], ["pod"])],
     "reference_error": False, "expect_no_calls": False},
    {"name": "Registry is not empty and no error for bytes", "src": "metrics_module_test.go:476-514",
     "prior": [_DC, mco("drop_bytes", ["ip"]), _FC, mco("forward_bytes", ["ip"])], "current_spec": None,
     "spec": [mco("drop_count", ["ip", "pod"], ["pod"]), mco("drop_bytes", ["ip"]),
              mco("forward_count", ["ip", "pod"], ["pod"]), mco("forward_bytes", ["ip"])],
     "reference_error": False, "expect_no_calls": False},
    {"name": "Registry is not empty and error for invalid name", "src": "metrics_module_test.go:515-553",
     "prior": [_DC, mco("drop_bytes", ["ip"]), _FC, mco("forward_bytes", ["ip"])], "current_spec": None,
     "spec": [mco("drop_hello", ["ip", "pod"], ["pod"]), mco("drop_bytes", ["ip"]),
              mco("forward_count", ["ip", "pod"], ["pod"]), mco("forward_hi", ["ip"])],
     "reference_error": False, "expect_no_calls": False},
    {"name": "Expect no change for spec the same", "src": "metrics_module_test.go:554-587",
     "prior": [_DC], "current_spec": [_DC], "spec": [_DC],
     "reference_error": False, "expect_no_calls": True},
]

# docs/06-Troubleshooting/basic-metrics.md:86-124: a scrape of the agent's /metrics (the
# basic registry: GaugeVecs through the same client_golang text encoder as the advanced
# registry), as printed by the reference's docs -- families, Help strings, label pairs
# and float64 values as data, and the exact text they render to
_G = "gauge"
kat["exposition_sample"] = {
    "src": "docs/06-Troubleshooting/basic-metrics.md:86-124",
    "families": {
        "retina_forward_bytes": [_G, "Total forwarded bytes"],
        "retina_forward_count": [_G, "Total forwarded packets"],
        "retina_interface_stats": [_G, "Interface Statistics"],
        "retina_ip_connection_stats": [_G, "IP connections Statistics"],
        "retina_tcp_connection_remote": [_G, "number of active TCP connections by remote address"],
        "retina_tcp_connection_stats": [_G, "TCP connections Statistics"],
        "retina_tcp_state": [_G, "number of active TCP connections by state"],
        "retina_udp_connection_stats": [_G, "UDP connections Statistics"],
    },
    # listed out of order on purpose: the encoder sorts families, metrics and label pairs
    "series": [
        ["retina_tcp_state", {"state": "TIME_WAIT"}, 89],
        ["retina_forward_count", {"direction": "ingress"}, 37254085],
        ["retina_forward_bytes", {"direction": "ingress"}, 23619602627],
        ["retina_forward_bytes", {"direction": "egress"}, 19064666952],
        ["retina_forward_count", {"direction": "egress"}, 43139614],
        ["retina_interface_stats", {"statistic_name": "vf_rx_packets", "interface_name": "eth0"}, 12948929],
        ["retina_interface_stats", {"statistic_name": "vf_rx_bytes", "interface_name": "eth0"}, 12679472174],
        ["retina_ip_connection_stats", {"statistic_name": "OutOctets"}, 27768258214],
        ["retina_ip_connection_stats", {"statistic_name": "InECT0Pkts"}, 34713],
        ["retina_ip_connection_stats", {"statistic_name": "InOctets"}, 16718610902],
        ["retina_ip_connection_stats", {"statistic_name": "InNoECTPkts"}, 38893357],
        ["retina_tcp_connection_remote", {"port": "7070", "address": "10.224.0.105"}, 1],
        ["retina_tcp_connection_remote", {"port": "0", "address": "0.0.0.0"}, 8],
        ["retina_tcp_connection_remote", {"port": "443", "address": "10.0.0.1"}, 1],
        ["retina_tcp_connection_stats", {"statistic_name": "DelayedACKLocked"}, 107],
        ["retina_tcp_state", {"state": "SYN_SENT"}, 1],
        ["retina_tcp_state", {"state": "CLOSE_WAIT"}, 1],
        ["retina_tcp_state", {"state": "LISTEN"}, 8],
        ["retina_tcp_state", {"state": "ESTABLISHED"}, 16],
        ["retina_tcp_state", {"state": "FIN_WAIT2"}, 1],
        ["retina_tcp_state", {"state": "FIN_WAIT1"}, 1],
        ["retina_tcp_state", {"state": "LAST_ACK"}, 1],
        ["retina_udp_connection_stats", {"statistic_name": "ACTIVE"}, 5],
    ],
    "text": [
        '# HELP retina_forward_bytes Total forwarded bytes',
        '# TYPE retina_forward_bytes gauge',
        'retina_forward_bytes{direction="egress"} 1.9064666952e+10',
        'retina_forward_bytes{direction="ingress"} 2.3619602627e+10',
        '# HELP retina_forward_count Total forwarded packets',
        '# TYPE retina_forward_count gauge',
        'retina_forward_count{direction="egress"} 4.3139614e+07',
        'retina_forward_count{direction="ingress"} 3.7254085e+07',
        '# HELP retina_interface_stats Interface Statistics',
        '# TYPE retina_interface_stats gauge',
        'retina_interface_stats{interface_name="eth0",statistic_name="vf_rx_bytes"} 1.2679472174e+10',
        'retina_interface_stats{interface_name="eth0",statistic_name="vf_rx_packets"} 1.2948929e+07',
        '# HELP retina_ip_connection_stats IP connections Statistics',
        '# TYPE retina_ip_connection_stats gauge',
        'retina_ip_connection_stats{statistic_name="InECT0Pkts"} 34713',
        'retina_ip_connection_stats{statistic_name="InNoECTPkts"} 3.8893357e+07',
        'retina_ip_connection_stats{statistic_name="InOctets"} 1.6718610902e+10',
        'retina_ip_connection_stats{statistic_name="OutOctets"} 2.7768258214e+10',
        '# HELP retina_tcp_connection_remote number of active TCP connections by remote address',
        '# TYPE retina_tcp_connection_remote gauge',
        'retina_tcp_connection_remote{address="0.0.0.0",port="0"} 8',
        'retina_tcp_connection_remote{address="10.0.0.1",port="443"} 1',
        'retina_tcp_connection_remote{address="10.224.0.105",port="7070"} 1',
        '# HELP retina_tcp_connection_stats TCP connections Statistics',
        '# TYPE retina_tcp_connection_stats gauge',
        'retina_tcp_connection_stats{statistic_name="DelayedACKLocked"} 107',
        '# HELP retina_tcp_state number of active TCP connections by state',
        '# TYPE retina_tcp_state gauge',
        'retina_tcp_state{state="CLOSE_WAIT"} 1',
        'retina_tcp_state{state="ESTABLISHED"} 16',
        'retina_tcp_state{state="FIN_WAIT1"} 1',
        'retina_tcp_state{state="FIN_WAIT2"} 1',
        'retina_tcp_state{state="LAST_ACK"} 1',
        'retina_tcp_state{state="LISTEN"} 8',
        'retina_tcp_state{state="SYN_SENT"} 1',
        'retina_tcp_state{state="TIME_WAIT"} 89',
        '# HELP retina_udp_connection_stats UDP connections Statistics',
        '# TYPE retina_udp_connection_stats gauge',
        'retina_udp_connection_stats{statistic_name="ACTIVE"} 5',
    ],
}

# pkg/utils/flow_utils.go:75-91 and dns.go:222: the Go identifiers of cilium's
# flow.TrafficDirection values.  protoc-gen-go names a constant <Enum>_<proto value name>,
# and the enum's String() (the metrics' direction label, forward.go:116) returns that value
# name, so the identifiers fix the label text
kat["traffic_direction_identifiers"] = {
    "src": "pkg/utils/flow_utils.go:75-91",
    "identifiers": ["TrafficDirection_EGRESS", "TrafficDirection_INGRESS",
                    "TrafficDirection_TRAFFIC_DIRECTION_UNKNOWN"],
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kat.json")
    with open(out, "w") as f:
        json.dump(kat, f, indent=1, sort_keys=True)
    print("wrote", out, len(kat["metric_objects"]), "metric-object cases")
