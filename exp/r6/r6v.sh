#!/bin/bash
# wide-kernel list diagnostics (c4-remote): full lists per workgroup
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
GPUAGG_LIB=$PWD/exp/r6/lib_ldiag.so timeout -k 10 300 python bench.py --config c4-remote --steps 3 --warmup 1 --settle-ms 0 \
  --no-cpu-baseline --no-host-fed --no-production --no-scrape > gpurun_out/r6v_diag.log 2>&1
