#!/bin/bash
# search-first hot-key cache (doorkeeper only with a free way): tests, A/B vs 200b22fb
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py -k "hot_key or c4_remote" > gpurun_out/r6z3_pytest.log 2>&1 || exit $?
bash exp/r6/ab.sh r6z3_ab c4-remote tree exp/r6/lib_200b.so || exit $?
bash exp/r6/ab.sh r6z3_ab1 c1 tree exp/r6/lib_200b.so
