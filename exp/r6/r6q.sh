#!/bin/bash
# read-first fold probes: wide / remote parity tests, then A/B vs build d45bc644
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py -k "hot_key or c4_remote" > gpurun_out/r6q_pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > gpurun_out/r6q_pytest2.log 2>&1 || exit $?
bash exp/r6/ab.sh r6q_ab c4-remote tree exp/r6/lib_d45b.so || exit $?
bash exp/r6/ab.sh r6q_ab1 c1 tree exp/r6/lib_d45b.so
