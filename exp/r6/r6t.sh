#!/bin/bash
# wide-list fold diagnostics: the fullest list per launch (c4-remote)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
GPUAGG_LIB=$PWD/exp/r6/lib_fprint.so timeout -k 10 300 python bench.py --config c4-remote --steps 10 --warmup 2 --settle-ms 0 \
  --no-cpu-baseline --no-host-fed --no-production --no-scrape > gpurun_out/r6t_bench.log 2>&1
