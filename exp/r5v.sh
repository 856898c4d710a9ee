#!/bin/bash
# round 5 probe: c4-remote / C1 bench lines of the round-4 build (exp/lib_r4.so), the build
# before the 2^11-slot wide fold segments (exp/lib_base.so) and the tree, interleaved on one box
cd "$(dirname "$0")/.."
export BENCH_CACHE=/tmp/benchcache_r5v
for cfg in c4-remote c1; do
  for lib in exp/lib_r4.so exp/lib_base.so "" exp/lib_r4.so exp/lib_base.so ""; do
    GPUAGG_LIB=${lib:+$PWD/$lib} timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-host-fed \
      --no-production --no-scrape > gpurun_out/r5v_one.json 2>> gpurun_out/r5v.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/r5v_one.json')); r=d['roofline']; print(json.dumps({'lib': sys.argv[1], 'cfg': sys.argv[2], 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'other_ms': r['other_kernels_ms']}))" "${lib:-tree}" $cfg >> gpurun_out/r5v.jsonl
  done
done
