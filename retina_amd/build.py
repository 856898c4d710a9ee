"""In-tree build of the gfx950 engine library (``retina_amd/libgpuagg.so``).

Plain ``hipcc`` invocations (no cmake/ninja): the kernels translation unit is built
for ``--offload-arch=gfx950`` only, the host runtime as ordinary C++; both are linked
into one shared library whose exported symbols are exactly ``include/gpuagg.h``.
"""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgpuagg.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["gpuagg_kernels.hip", "gpuagg_decode.hip", "gpuagg_latency.hip", "gpuagg_hubble.hip",
           "gpuagg_runtime.cpp"]
HEADERS = ["gpuagg_internal.h", "gpuagg_launch.h", os.path.join("..", "..", "include", "gpuagg.h")]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def _run(cmd) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("build failed: " + " ".join(cmd))


def build(force: bool = False, verbose: bool = False) -> str:
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    if not force and _newer(LIB, deps):
        return LIB
    objs = []
    common = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-I", CSRC,
              "-I", os.path.join(ROOT, "include")]
    hdrs = [os.path.join(CSRC, h) for h in HEADERS]
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(CSRC, os.path.splitext(s)[0] + ".o")
        objs.append(obj)
        if not force and _newer(obj, [src] + hdrs):  # up to date: reuse the object
            continue
        if s.endswith(".hip"):
            cmd = [HIPCC, "--offload-arch=" + ARCH, "-munsafe-fp-atomics"] + common + ["-c", src, "-o", obj]
        else:
            cmd = [HIPCC] + common + ["-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include",
                                      "-x", "c++", "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
    tmp = LIB + ".tmp"
    _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs
         + ["-Wl,--version-script=" + os.path.join(CSRC, "gpuagg.map")])
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
