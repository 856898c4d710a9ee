#!/bin/bash
# narrow (24-byte) wide-list entries: remote / wide parity tests, then A/B vs build d45bc644
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_dist.py > gpurun_out/r6n_pytest.log 2>&1 || exit $?
bash exp/r6/ab.sh r6n_ab c4-remote tree exp/r6/lib_d45b.so || exit $?
bash exp/r6/ab.sh r6n_ab1 c1 tree exp/r6/lib_d45b.so
