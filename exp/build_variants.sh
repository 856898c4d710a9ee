#!/bin/bash
# Diagnostic builds of the engine library with -D experiment switches (not product code).
set -e
cd "$(dirname "$0")/.."
C=retina_amd/csrc
for v in "$@"; do
  name=${v:-base}
  D=""; [ -n "$v" ] && D="-D$v"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics -O3 -fPIC -std=c++17 -I $C -I include $D -c $C/gpuagg_kernels.hip -o /tmp/k_$name.o &
done
wait
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -I $C -I include -D__HIP_PLATFORM_AMD__ -I /opt/rocm/include -x c++ -c $C/gpuagg_runtime.cpp -o /tmp/rt.o
for v in "$@"; do
  name=${v:-base}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o exp/lib_$name.so /tmp/k_$name.o /tmp/rt.o -Wl,--version-script=$C/gpuagg.map
done
ls -la exp/*.so
