#!/bin/bash
# round 6, call b: secondary-bound microbenchmarks; C3 with the scatter-only sketch timing
cd "$(dirname "$0")/../.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 ./scripts/mbb > $OUT/r6b_bounds.jsonl 2> $OUT/r6b_bounds.err || exit $?
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-fed --no-production \
  --no-scrape > $OUT/r6b_bench_c3.json 2> $OUT/r6b_bench_c3.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r6b_prof_c3 -o run \
  -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-fed --no-production --no-scrape \
  > $OUT/r6b_prof_c3.log 2>&1 || exit $?
find $OUT/r6b_prof_c3 -name "*kernel_stats.csv" -exec cp {} $OUT/r6b_c3_kernel_stats.csv \;
