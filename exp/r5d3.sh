#!/bin/bash
# round 5: the driver's default command at the final build, twice
cd "$(dirname "$0")/.."
for k in 1; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5d3_bench_default_$k.json 2> gpurun_out/r5d3_default.err || exit $?
done
