#!/bin/bash
# round 5 probe: gpuagg_sync without the per-sync timing drain and blocking counter copies
# (tree) vs build d4ffb926 (exp/lib_prev.so): the driver's command, interleaved
cd "$(dirname "$0")/.."
export BENCH_CACHE=/tmp/benchcache_r5z
for lib in exp/lib_prev.so "" exp/lib_prev.so "" exp/lib_prev.so ""; do
  GPUAGG_LIB=${lib:+$PWD/$lib} timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed \
    --no-production --no-scrape > gpurun_out/r5z_one.json 2>> gpurun_out/r5z.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r5z_one.json')); r=d['roofline']; print(json.dumps({'lib': sys.argv[1], 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'other_ms': r['other_kernels_ms']}))" "${lib:-tree}" >> gpurun_out/r5z.jsonl
done
