#!/bin/bash
# round 5 probe: deferred folds with the spill-window fold on a second stream beside the
# segment fold (tree) vs build 5b4a29a3 (exp/lib_prev.so): C5 / DNS / deferred-fold GPU
# tests, then C5 bench lines interleaved
cd "$(dirname "$0")/.."
export BENCH_CACHE=/tmp/benchcache_r5fj
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "c5 or dns or deferred or fold or lifecycle or scale" > gpurun_out/r5fj_pytest.log 2>&1 || exit $?
for lib in exp/lib_prev.so "" exp/lib_prev.so "" exp/lib_prev.so ""; do
  GPUAGG_LIB=${lib:+$PWD/$lib} timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-host-fed \
    --no-production --no-scrape > gpurun_out/r5fj_one.json 2>> gpurun_out/r5fj.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r5fj_one.json')); r=d['roofline']; print(json.dumps({'lib': sys.argv[1], 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'other_ms': r['other_kernels_ms']}))" "${lib:-tree}" >> gpurun_out/r5fj.jsonl
done
