"""CPU-side checks of the C-ABI library: it builds, loads, exports exactly what
include/gpuagg.h declares, and refuses to run without a gfx950 device (no fallback)."""

import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gpuagg.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"\b(gpuagg_[a-z_]+)\s*\(", txt))


@pytest.fixture(scope="module")
def lib():
    from retina_amd import build
    build.build()
    from retina_amd import _abi
    return _abi.load()


def test_exports_match_header(lib):
    nm = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "retina_amd", "libgpuagg.so")],
                        stdout=subprocess.PIPE, text=True, check=True).stdout
    exported = {l.split()[-1] for l in nm.splitlines() if l.split() and l.split()[-1].startswith("gpuagg_")}
    assert exported == declared_symbols()


def test_binding_covers_header():
    from retina_amd import _abi
    assert {s[0] for s in _abi.SIGNATURES} == declared_symbols()


def test_create_without_gpu_fails_loudly(lib):
    from retina_amd import _abi, GpuAgg, GpuAggError
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    with pytest.raises(GpuAggError) as e:
        GpuAgg(device=0)
    assert e.value.code == _abi.EDEVICE


def test_bad_config_rejected(lib):
    from retina_amd import _abi
    cfg = _abi.Config(999, 0, 0, 16, 16, 10, 0, 0, 0)
    h = C.c_void_p()
    assert lib.gpuagg_create(C.byref(cfg), C.byref(h)) == _abi.EINVAL
    assert lib.gpuagg_last_error(None) == b"null ctx"
