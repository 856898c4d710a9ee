#!/bin/bash
# per-segment fold decision: tests, A/B vs 4a7e241 and thr 3/4
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_dist.py > gpurun_out/r6w_pytest.log 2>&1 || exit $?
bash exp/r6/ab.sh r6w_ab c4-remote tree exp/r6/lib_thr34.so exp/r6/lib_4a7e.so || exit $?
bash exp/r6/ab.sh r6w_ab1 c1 tree exp/r6/lib_4a7e.so
