"""The Go plugin's known-answer test (go/pkg/gpuagg/records_linux_test.go: PacketRecord,
DropRecord and ipv4LE against the oracle's decode and net.ParseIP's IPv4 rules) is the
file tests/golden/make_go_vectors.py writes -- so the vectors a maintainer runs with
`go test -tags gpuagg` are the oracle's, not the Go code's own output."""
import importlib.util
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def _gen():
    spec = importlib.util.spec_from_file_location("make_go_vectors", os.path.join(HERE, "golden", "make_go_vectors.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_go_vector_file_is_current():
    m = _gen()
    with open(m.OUT) as f:
        assert f.read() == m.render(), "regenerate: python tests/golden/make_go_vectors.py"


def test_go_vectors_cover_edge_rows():
    m = _gen()
    prow, pb, drow, db = m.vectors()
    assert (pb.meta >> 8 & 0xFF == 255).any()        # a traffic direction no metric consumes
    assert (prow["obs"] > 3).any()                    # an unknown observation point
    assert (db.meta >> 8 & 0xFF == 255).any()        # a drop type past the enum
    assert sum(m.ipv4_le(s) is None for s in m.IPV4_CASES) >= 10
