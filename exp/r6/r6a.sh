#!/bin/bash
# round 6, call a: the multi-rank bench path on one GPU + the driver's N=1 command
cd "$(dirname "$0")/../.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_bench_ranks.py -m gpu -x -v --timeout 280 --timeout-method thread \
  > $OUT/r6a_pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r6a_bench_c2.json 2> $OUT/r6a_bench_c2.err || exit $?
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-scrape --check-merge \
  > $OUT/r6a_bench_c2_gloo2.json 2> $OUT/r6a_bench_c2_gloo2.err || exit $?
