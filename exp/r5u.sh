#!/bin/bash
# round 5 probe: c4-remote wide-list fold threshold cap/4, cap*3/4 (product cap/2) and 64 GiB
# of lists, at the 2^11-slot fold segments; then c4-remote and C1 bench lines of the tree
cd "$(dirname "$0")/.."
export BENCH_CACHE=/tmp/benchcache_r5u
for lib in "" exp/lib_thr4.so exp/lib_thr34.so exp/lib_64g.so ""; do
  GPUAGG_LIB=${lib:+$PWD/$lib} ABLATE_ONLY=c4r timeout -k 10 300 python scripts/ablate.py >> gpurun_out/r5u_c4r.jsonl 2>> gpurun_out/r5u.err || exit $?
done
for cfg in c4-remote c1; do
  timeout -k 10 600 python bench.py --config $cfg > gpurun_out/r5u_bench_$cfg.json 2>> gpurun_out/r5u.err || exit $?
done
