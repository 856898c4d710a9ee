#!/bin/bash
# round 5 probe: wide-key probe segments of 2^11 slots in pairs under 4096 list segments
# (tree; two fold workgroups per CU, lists as before) vs the 2^12-slot build (exp/lib_base.so):
# wide / sparse / remote GPU tests, then c4-remote and C1 bench lines interleaved
cd "$(dirname "$0")/.."
export BENCH_CACHE=/tmp/benchcache_r5w
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "remote or wide or sparse or scale or c4" > gpurun_out/r5w_pytest.log 2>&1 || exit $?
for cfg in c4-remote c1; do
  for lib in exp/lib_base.so "" exp/lib_base.so ""; do
    GPUAGG_LIB=${lib:+$PWD/$lib} timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-host-fed \
      --no-production --no-scrape > gpurun_out/r5w_one.json 2>> gpurun_out/r5w.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/r5w_one.json')); r=d['roofline']; print(json.dumps({'lib': sys.argv[1], 'cfg': sys.argv[2], 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'other_ms': r['other_kernels_ms']}))" "${lib:-tree}" $cfg >> gpurun_out/r5w.jsonl
  done
done
