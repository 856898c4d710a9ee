#!/bin/bash
# round 5 probe: c4-remote wide-list fold threshold (product sp_cap/2, 7/8, never until sync)
cd "$(dirname "$0")/.."
for lib in "" exp/lib_wthr_78.so exp/lib_wthr_never.so; do
  GPUAGG_LIB=${lib:+$PWD/$lib} ABLATE_ONLY=c4r timeout -k 10 300 python scripts/ablate.py >> gpurun_out/r5h_c4r.jsonl 2>> gpurun_out/r5h.err || exit $?
done
