#!/bin/bash
# round 5 probe: wide-key fold segments of 2^11 slots with u16 list counters (tree) vs the
# committed 2^12-slot build (exp/lib_base.so); parity tests of the wide-list paths first
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "remote or wide or sparse or scale or c4" > gpurun_out/r5t_pytest.log 2>&1 || exit $?
for lib in exp/lib_base.so "" exp/lib_base.so ""; do
  GPUAGG_LIB=${lib:+$PWD/$lib} ABLATE_ONLY=c4r timeout -k 10 300 python scripts/ablate.py >> gpurun_out/r5t_c4r.jsonl 2>> gpurun_out/r5t.err || exit $?
done
