#!/bin/bash
# 16-byte fold segment loads / stores + read-first compact fold: tests, then A/B vs 4a7e241
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py -k "hot_key or c4_remote" tests/test_dns_retire.py tests/test_gpu_parity.py > gpurun_out/r6r_pytest.log 2>&1 || exit $?
bash exp/r6/ab.sh r6r_ab c4-remote tree exp/r6/lib_4a7e.so || exit $?
bash exp/r6/ab.sh r6r_ab5 c5 tree exp/r6/lib_4a7e.so
