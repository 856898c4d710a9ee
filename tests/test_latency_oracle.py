"""The latency restatement (oracle/latency.py) against the reference's own test,
pkg/module/metrics/latency_test.go:83-170 (TestProcessFlow): a SYN / SYN+ACK pair 1 ms
apart observes 1 ms on both histograms; a SYN / ACK pair observes only the latency
histogram; an unanswered request counts one no_response once the TTL has passed."""

from oracle import latency as L
from oracle import oracle as O


def _flow(t, src, dst, sport, dport, obs, syn, ack, tcp_id):
    f = O.to_flow(src, dst, sport, dport, 6, obs, 0)
    f.time_ns = t
    f.extensions = O.RetinaMetadata(tcp_id=tcp_id)
    O.add_tcp_flags(f, syn, ack, 0, 0, 0, 0)
    return f


def test_reference_process_flow_cases():
    api, node = "1.1.1.1", "2.2.2.2"
    m = L.LatencyMetrics({L.LATENCY, L.HANDSHAKE, L.NO_RESPONSE})
    m.add_ips([api])
    t1 = 1_700_000_000_500_000_000  # mid-second, as the reference test assumes
    t2 = t1 + 1_000_000
    # case 1: TCP handshake
    m.process_flow(_flow(t1, api, node, 80, 443, 3, 1, 0, 1234))
    m.process_flow(_flow(t2, node, api, 443, 80, 2, 1, 1, 1234))
    # case 2: existing connection
    m.process_flow(_flow(t1, api, node, 80, 443, 3, 1, 0, 1234))
    m.process_flow(_flow(t2, node, api, 443, 80, 2, 0, 1, 1234))
    # case 3: no reply; one second later the entry has expired
    m.process_flow(_flow(t1, api, node, 80, 443, 3, 1, 0, 1234))
    m.finish(now_ns=t2 + 1_000_000_000)
    assert m.latency.count == 2 and m.latency.total == 2.0
    assert m.handshake.count == 1 and m.handshake.total == 1.0
    assert m.no_response == 1
    # 1 ms lands in the le="1" bucket (upper bounds 0, 0.5, 1, ...)
    assert m.latency.buckets[2] == 2
    text = L.render(m)
    assert 'networkobservability_adv_node_apiserver_latency_bucket{le="1"} 2' in text
    assert 'networkobservability_adv_node_apiserver_no_response{no_response="no_response"} 1' in text


def test_filters_and_second_wrap():
    api, node = "1.1.1.1", "2.2.2.2"
    m = L.LatencyMetrics({L.LATENCY})
    m.add_ips([api])
    t = 5_999_999_000  # 1 ms before a second boundary
    # tcp id 0 and non-apiserver traffic are ignored
    m.process_flow(_flow(t, api, node, 1, 2, 3, 1, 0, 0))
    m.process_flow(_flow(t, "3.3.3.3", node, 1, 2, 3, 1, 0, 7))
    # a pair straddling the second boundary: Nanos-only arithmetic gives a negative latency
    m.process_flow(_flow(t, node, api, 1000, 443, 3, 1, 0, 9))
    m.process_flow(_flow(t + 2_000_000, api, node, 443, 1000, 2, 1, 1, 9))
    assert m.latency.count == 1 and m.latency.total == -998.0
    assert m.latency.buckets[0] == 1
    assert m.no_response is None and not m.cache  # ignored flows never entered


def test_go_round_half_away_from_zero():
    assert L.go_round(0.5) == 1.0 and L.go_round(-0.5) == -1.0 and L.go_round(1.4999) == 1.0
