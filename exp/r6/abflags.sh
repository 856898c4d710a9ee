#!/bin/bash
# A/B of engine flags on the product library (GPUAGG_BENCH_FLAGS), interleaved 3 rounds.
#   bash exp/r6/abflags.sh TAG CONFIG FLAGS...
cd "$(dirname "$0")/../.."
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out
mkdir -p $OUT
export BENCH_CACHE=/tmp/benchcache_$TAG
for round in 1 2 3; do
  for fl in "$@"; do
    GPUAGG_BENCH_FLAGS=$fl timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed \
      --no-production --no-scrape > $OUT/${TAG}_one.json 2>> $OUT/${TAG}.err || exit $?
    python -c "import json,sys; d=json.loads(open('$OUT/${TAG}_one.json').read().strip().splitlines()[-1]); r=d['roofline']; print(json.dumps({'flags': sys.argv[1], 'round': int(sys.argv[2]), 'ms_per_step': d['ms_per_step'], 'kernel': r['kernel'], 'kernel_ms': r['kernel_ms'], 'frac': r['frac'], 'other_ms': r['other_kernels_ms']}))" "$fl" $round >> $OUT/${TAG}.jsonl
  done
done
