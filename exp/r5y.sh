#!/bin/bash
# round 5: settle launches in groups of 8 (bench.py) -- C1 bench + rocprof agreement, C5
# rocprof, and the driver's default command
cd "$(dirname "$0")/.."
bash scripts/gpu_check.sh r5y bench:c1 prof:c1 prof:c5 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5y_bench_default.json 2> gpurun_out/r5y_default.err || exit $?
