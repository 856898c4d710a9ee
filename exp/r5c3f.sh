#!/bin/bash
# round 5 probe: C3's cms_fold beside the HLL split + fold on a second stream
# (exp/lib_c3fork.so, exp/patch_c3_fork.py) vs the final build: sketch GPU tests with the
# probe library, then C3 bench lines interleaved
cd "$(dirname "$0")/.."
export BENCH_CACHE=/tmp/benchcache_r5c3f
GPUAGG_LIB=$PWD/exp/lib_c3fork.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sketch.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r5c3f_pytest.log 2>&1 || exit $?
for lib in "" exp/lib_c3fork.so "" exp/lib_c3fork.so "" exp/lib_c3fork.so; do
  GPUAGG_LIB=${lib:+$PWD/$lib} timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-host-fed \
    --no-production --no-scrape > gpurun_out/r5c3f_one.json 2>> gpurun_out/r5c3f.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/r5c3f_one.json')); r=d['roofline']; print(json.dumps({'lib': sys.argv[1], 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'other_ms': r['other_kernels_ms']}))" "${lib:-final}" >> gpurun_out/r5c3f.jsonl
done
