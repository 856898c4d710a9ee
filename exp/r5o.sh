#!/bin/bash
# round 5 probe: C2 / C4 fold partitions per window
cd "$(dirname "$0")/.."
for lib in "" exp/lib_fp4.so exp/lib_fp8.so exp/lib_fp12.so; do
  GPUAGG_LIB=${lib:+$PWD/$lib} ABLATE_ONLY=c2,c4-zipf timeout -k 10 300 python scripts/ablate.py >> gpurun_out/r5o_c2.jsonl 2>> gpurun_out/r5o.err || exit $?
done
