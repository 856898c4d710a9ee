"""The Go plugin (go/pkg/gpuagg) has no compiler here: check its source statically.

`test_go_package_static_clean` is the gate on the real tree (round 4 shipped a package
that declared `ipv4LE` in two files of one build set); the other tests pin each check on
a small synthetic package, so a check that silently stopped firing would show.
"""
import os
import textwrap

import pytest

from tests import go_static as gs


def test_go_package_static_clean():
    errs = gs.all_errors()
    assert errs == [], "\n".join(errs)


def test_go_package_implements_enricher_interface():
    # pkg/enricher/types.go:12-16: Run(), Write(*v1.Event), ExportReader() *container.RingReader
    files = gs.load_package()
    meths = {(rt, nm) for f in files for rt, nm, _ in f.methods}
    for m in ("Run", "Write", "ExportReader"):
        assert ("Enricher", m) in meths
    # pkg/plugin/registry/registry.go:16-34: the Plugin interface
    for m in ("Name", "Generate", "Compile", "Init", "Start", "Stop", "SetupChannel"):
        assert ("gpuAgg", m) in meths


def _pkg(tmp_path, files: dict) -> list:
    d = tmp_path / "pkg"
    d.mkdir()
    for name, src in files.items():
        (d / name).write_text(textwrap.dedent(src))
    return gs.load_package(str(d))


HDR = """\
//go:build linux && gpuagg

package p
"""


def test_duplicate_across_files_is_caught(tmp_path):
    fs = _pkg(tmp_path, {
        "a.go": HDR + "func ipv4LE(s string) (uint32, bool) { return 0, false }\n",
        "b.go": HDR + "func ipv4LE(s string) (uint32, bool) { return 1, true }\n",
    })
    errs = gs.duplicate_declarations(fs)
    assert len(errs) == 1 and "ipv4LE redeclared" in errs[0]


def test_duplicate_in_other_build_set_is_fine(tmp_path):
    fs = _pkg(tmp_path, {
        "a.go": HDR + "func f() {}\n",
        "b.go": "//go:build !linux\n\npackage p\n\nfunc f() {}\n",
    })
    assert gs.duplicate_declarations(fs) == []


def test_grouped_const_and_method_duplicates(tmp_path):
    fs = _pkg(tmp_path, {
        "a.go": HDR + "const (\n\tx = 1\n\ty = 2\n)\n\ntype T struct{}\n\nfunc (t *T) M() {}\n",
        "b.go": HDR + "var y = 3\n\nfunc (t T) M() {}\n",
    })
    errs = gs.duplicate_declarations(fs)
    assert any("y redeclared" in e for e in errs)
    assert any("method T.M redeclared" in e for e in errs)


def test_unused_and_missing_imports(tmp_path):
    fs = _pkg(tmp_path, {
        "a.go": HDR + 'import (\n\t"net"\n\t"strings"\n)\n\nfunc f(s string) string { return strings.ToLower(s) }\n'
                      "func g(b []byte) uint32 { return binary.LittleEndian.Uint32(b) }\n",
    })
    errs = gs.import_errors(fs)
    assert any('"net" imported and not used' in e for e in errs)
    assert any("undefined: binary" in e for e in errs)
    assert not any("strings" in e for e in errs)


def test_cgo_names_checked_against_header(tmp_path, monkeypatch):
    fs = _pkg(tmp_path, {
        "a.go": HDR + '/*\n#include "gpuagg.h"\n*/\nimport "C"\n\n'
                      "func f() { C.gpuagg_sync(nil); C.gpuagg_nope(nil); _ = C.sizeof_gpuagg_record; "
                      "_ = C.GPUAGG_OK; _ = C.CString(\"\") }\n",
    })
    errs = gs.cgo_errors(fs)
    assert len(errs) == 1 and "C.gpuagg_nope" in errs[0]


def test_record_layout_drift_is_caught(tmp_path):
    good = "type Record struct {\n\tSrcIP, DstIP, Bytes, Meta, Ports, DNSID uint32\n\tTcpID uint32\n\tTimeNs uint64\n}\n"
    assert gs.record_layout_errors(_pkg(tmp_path, {"a.go": HDR + good})) == []
    swapped = good.replace("Bytes, Meta", "Meta, Bytes")
    (tmp_path / "pkg" / "a.go").write_text(HDR + swapped)
    assert gs.record_layout_errors(gs.load_package(str(tmp_path / "pkg")))
    narrow = good.replace("TimeNs uint64", "TimeNs uint32")
    (tmp_path / "pkg" / "a.go").write_text(HDR + narrow)
    assert gs.record_layout_errors(gs.load_package(str(tmp_path / "pkg")))


def test_undefined_calls_are_caught(tmp_path):
    fs = _pkg(tmp_path, {
        "a.go": HDR + "type T struct{}\n\nfunc (t *T) run() {}\n\n"
                      "func f(t *T, fn func()) uint32 { t.run(); t.walk(); fn(); x := helper; _ = x; return b2u(true) }\n",
    })
    errs = gs.undefined_calls(fs)
    assert any("undefined: b2u" in e for e in errs)
    assert any(".walk() is no method" in e for e in errs)
    assert not any("run" in e or "fn" in e for e in errs)


def test_integration_snippet_check(tmp_path):
    fs = gs.load_package()
    md = tmp_path / "I.md"
    md.write_text("x\n```go\nrec := gpuagg.Record{Meta: b2u(ev.IsReply) << 27}\n"
                  "gpuagg.NoSuchThing(rec)\nn := len(rec.Meta)\n```\n")
    errs = gs.snippet_errors(str(md), fs)
    assert any("b2u()" in e for e in errs)
    assert any("gpuagg.NoSuchThing" in e for e in errs)
    assert not any("len" in e for e in errs)


@pytest.mark.parametrize("name", ["enricher_linux.go", "gpuagg_linux.go"])
def test_every_file_has_the_build_tag(name):
    f = gs.parse_go(os.path.join(gs.GO_PKG, name))
    assert f.build == "linux && gpuagg" and f.package == "gpuagg"


def test_receiver_selectors_are_checked(tmp_path):
    fs = _pkg(tmp_path, {
        "a.go": HDR + "type T struct {\n\tmu sync.Mutex\n\ta, b int\n\t*Embedded\n}\n\n"
                      "func (t *T) f() int { t.mu.Lock(); t.g(); return t.a + t.b + t.rawBuf + t.Embedded.x }\n\n"
                      "func (t *T) g() {}\n",
    })
    errs = gs.selector_errors(fs)
    assert len(errs) == 1 and "t.rawBuf undefined" in errs[0]
