#!/bin/bash
# round 5 probe: C5 with a 4-iteration radix prefix loop
cd "$(dirname "$0")/.."
for lib in "" exp/lib_radix4.so; do
  GPUAGG_LIB=${lib:+$PWD/$lib} ABLATE_N=1000000 ABLATE_ONLY=c5,c5-retrans timeout -k 10 240 python scripts/ablate.py >> gpurun_out/r5n_c5.jsonl 2>> gpurun_out/r5n.err || exit $?
done
