#!/bin/bash
cd "$(dirname "$0")/../.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "c2 or packed or parity or deferred or c4" > $OUT/r6h_pytest.log 2>&1 || exit $?
bash exp/r6/ab.sh r6h_ab c2 exp/lib_base.so tree
bash exp/r6/ab.sh r6h_ab4 c4 exp/lib_base.so tree
