#!/bin/bash
# round 5 probe: full-size tier-1 spill fold + reduce on a second stream beside the next
# launch's kernel (double-buffered lists; GPUAGG_TAIL_OVERLAP=0 keeps them on the ctx's
# stream): the whole GPU suite, then C2 / C4 / C3 bench lines interleaved
cd "$(dirname "$0")/.."
export BENCH_CACHE=/tmp/benchcache_r5tail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5tail_pytest.log 2>&1 || exit $?
for cfg in c2 c2 c2 c4 c3; do
  for ov in 0 1; do
    GPUAGG_TAIL_OVERLAP=$ov timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline \
      --no-host-fed --no-production --no-scrape > gpurun_out/r5tail_one.json 2>> gpurun_out/r5tail.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/r5tail_one.json')); r=d['roofline']; print(json.dumps({'overlap': int(sys.argv[1]), 'cfg': sys.argv[2], 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'other_ms': r['other_kernels_ms']}))" $ov $cfg >> gpurun_out/r5tail.jsonl
  done
done
