#!/bin/bash
# Diagnostic builds of the engine library with -D experiment switches (not product code).
# A variant "A+B" defines both A and B.
set -e
cd "$(dirname "$0")/.."
C=retina_amd/csrc
rm -f exp/lib_*.so
for v in "$@"; do
  name=${v:-base}
  D=""; for d in ${v//+/ }; do D="$D -D$d"; done
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics -O3 -fPIC -std=c++17 -I $C -I include $D -c $C/gpuagg_kernels.hip -o /tmp/k_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics -O3 -fPIC -std=c++17 -I $C -I include $D -c $C/gpuagg_decode.hip -o /tmp/d_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics -O3 -fPIC -std=c++17 -I $C -I include $D -c $C/gpuagg_latency.hip -o /tmp/l_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics -O3 -fPIC -std=c++17 -I $C -I include $D -c $C/gpuagg_hubble.hip -o /tmp/h_$name.o &&
    /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -I $C -I include $D -D__HIP_PLATFORM_AMD__ -I /opt/rocm/include -x c++ -c $C/gpuagg_runtime.cpp -o /tmp/rt_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o exp/lib_$name.so /tmp/k_$name.o /tmp/d_$name.o /tmp/l_$name.o /tmp/h_$name.o /tmp/rt_$name.o -Wl,--version-script=$C/gpuagg.map ) &
done
wait
ls -la exp/*.so
