#!/bin/bash
cd "$(dirname "$0")/../.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_dns_retire.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/r6c_pytest.log 2>&1 || exit $?
bash exp/r6/ab.sh r6c_ab c2 tree exp/lib_pf2.so exp/lib_np2.so exp/lib_pf2np2.so
