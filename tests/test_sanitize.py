"""Host sanitizers on the library's C++ side.

The host runtime, the raw feed (its thread pool, the two pinned stagings per context and
their hand-off) and the CPU backend's host threads are built with ASan + UBSan and with
TSan (retina_amd/build.py build_sanitized; the gfx950 objects are not instrumented: device
sanitizers are not available on this pool), and the CPU tests that drive them run in a
child python with the clang runtime preloaded and GPUAGG_LIB pointing at the sanitized
library.  Canaries (tests/sanitize/canary.cpp: a heap overflow, a data race) built and
loaded the same way show the tools are live, so a clean run means something.
scripts/sanitize.sh runs the whole CPU files; here a selection keeps the suite short."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (files, -k selection) per sanitizer: the threaded paths first
RUNS = {
    "asan": (["tests/test_cpu_shard.py", "tests/test_cpu_abi.py", "tests/test_cpu_backend.py"],
             "not parity_vs_oracle and not exposition_order_every_case and not large_families"),
    "tsan": (["tests/test_cpu_shard.py", "tests/test_cpu_backend.py"],
             "raw_feed or record_feed or shard or merge or concurrent or scrape_buffers or exposition_text "
             "or sketches or latency_matches or retire"),
}


def _env(kind, lib, log):
    from retina_amd import build
    env = dict(os.environ)
    env["LD_PRELOAD"] = build.sanitizer_runtime(kind)
    env["GPUAGG_LIB"] = lib
    if kind == "asan":
        # python and torch are not instrumented: their leaks are not ours
        env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:log_path=%s" % log
        env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1:log_path=%s" % log
    else:
        env["TSAN_OPTIONS"] = "report_signal_unsafe=0:halt_on_error=0:log_path=%s" % log
    return env


def _reports(log):
    d, base = os.path.dirname(log), os.path.basename(log)
    out = []
    for f in sorted(os.listdir(d)):
        if f.startswith(base + "."):
            out.append(open(os.path.join(d, f), errors="replace").read())
    return out


@pytest.fixture(scope="module", params=["asan", "tsan"])
def sanitized(request):
    from retina_amd import build
    kind = request.param
    return kind, build.build_sanitized(kind), build.build_canary(kind)


def test_canary_is_caught(sanitized, tmp_path):
    kind, _, canary = sanitized
    log = str(tmp_path / "canary")
    fn = "canary_overflow(0)" if kind == "asan" else "canary_race(200000)"
    p = subprocess.run([sys.executable, "-c", "import ctypes; ctypes.CDLL(%r).%s" % (canary, fn)],
                       env=_env(kind, canary, log), capture_output=True, text=True, timeout=120)
    text = "".join(_reports(log)) + p.stderr
    if kind == "asan":
        assert p.returncode != 0 and "heap-buffer-overflow" in text, text[-2000:]
    else:
        assert "ThreadSanitizer: data race" in text, text[-2000:]


def test_cpu_paths_clean(sanitized, tmp_path):
    kind, lib, _ = sanitized
    files, sel = RUNS[kind]
    log = str(tmp_path / kind)
    p = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                        "-k", sel] + files, env=_env(kind, lib, log), capture_output=True, text=True, cwd=ROOT,
                       timeout=1500)
    reports = _reports(log)
    assert not reports, "%s reports:\n%s" % (kind, reports[0][:6000])
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    assert " passed" in p.stdout
