#!/bin/bash
# 3-way hot-key cache: tests, fullest-list diagnostics, A/B vs 4a7e241 (2-way) and thr 3/4
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py -k "hot_key or c4_remote" > gpurun_out/r6u_pytest.log 2>&1 || exit $?
GPUAGG_LIB=$PWD/exp/r6/lib_fprint.so timeout -k 10 300 python bench.py --config c4-remote --steps 10 --warmup 2 --settle-ms 0 \
  --no-cpu-baseline --no-host-fed --no-production --no-scrape > gpurun_out/r6u_diag.log 2>&1 || exit $?
bash exp/r6/ab.sh r6u_ab c4-remote tree exp/r6/lib_thr34.so exp/r6/lib_4a7e.so || exit $?
bash exp/r6/ab.sh r6u_ab1 c1 tree exp/r6/lib_4a7e.so
