#!/bin/bash
# fold probe waits on a same-k0 key being published (tree); + balanced lanes and per-segment
# deferred folds (variant): wide tests on both, then A/B vs the final build 4afcbe50
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py -k "hot_key or c4_remote" > gpurun_out/r6z5_pytest.log 2>&1 || exit $?
GPUAGG_LIB=$PWD/exp/r6/lib_baldef.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py -k "hot_key or c4_remote" > gpurun_out/r6z5_pytest_baldef.log 2>&1 || exit $?
bash exp/r6/ab.sh r6z5_ab c4-remote exp/r6/lib_4afc.so tree exp/r6/lib_baldef.so || exit $?
bash exp/r6/ab.sh r6z5_ab1 c1 exp/r6/lib_4afc.so tree exp/r6/lib_baldef.so
