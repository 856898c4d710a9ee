"""The Hubble L3/L4 restatement (oracle/hubble.py): endpoint decode and summaries (CPU).
The reference has no test for this parser; the cases follow decoder_linux.go and
layer34/parser_linux.go line by line (parity of the cilium constants is unpinned)."""

from oracle import hubble as H
from oracle import oracle as O


def test_endpoint_decode_rules():
    ipc = {"10.0.0.1": H.IPCacheEntry(12345, 0, ["k8s:app=a"]), "10.0.0.2": H.IPCacheEntry(H.ID_HOST),
           "10.0.0.3": H.IPCacheEntry(H.ID_KUBE_APISERVER, 1)}
    meta = {0: ("pod-a", "ns-a"), 1: ("kube-apiserver", "default")}
    a = H.decode_endpoint(ipc, meta, "10.0.0.1")
    assert (a.id, a.identity, a.pod_name, a.namespace, a.labels) == (12345, 12345, "pod-a", "ns-a", ["k8s:app=a"])
    assert H.decode_endpoint(ipc, meta, "10.0.0.2").labels == ["reserved:host"]
    k = H.decode_endpoint(ipc, meta, "10.0.0.3")
    assert k.labels == ["reserved:kube-apiserver"] and k.pod_name == "kube-apiserver"
    w = H.decode_endpoint(ipc, meta, "8.8.8.8")  # not in the ipcache: World
    assert (w.identity, w.labels, w.pod_name) == (H.ID_WORLD, ["reserved:world"], "")


def test_summaries():
    f = O.to_flow("1.1.1.1", "2.2.2.2", 1, 2, 6, 3, 1)
    O.add_tcp_flags(f, 1, 1, 0, 0, 0, 0)
    assert H.summary(f) == (H.SUM_TCP, 0b10010, "TCP Flags: SYN:true ACK:true")
    assert H.render_summary(H.SUM_TCP, 0b10010) == "TCP Flags: SYN:true ACK:true"
    u = O.to_flow("1.1.1.1", "2.2.2.2", 1, 2, 17, 3, 1)
    assert H.summary(u)[2] == "UDP"
    d = O.drop_flow("1.1.1.1", "2.2.2.2", 1, 2, 6, 3, 100)
    assert H.summary(d)[2].startswith("Drop Reason: TCP_ACCEPT_BASIC\nNote: ")
    n = O.to_flow("1.1.1.1", "2.2.2.2", 1, 2, 6, 3, 1)  # TCP without flags: no summary
    assert H.summary(n) == (H.SUM_NONE, 0, "")
    assert H.dns_summary(O.DNS(rcode=0, query="bing.com", qtypes=["A"], ips=["1.1.1.1"]), "REQUEST") == \
        "DNS Query bing.com A"
