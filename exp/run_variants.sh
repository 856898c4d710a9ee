#!/bin/bash
# Runs scripts/ablate.py against each experiment library (GPU box).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lib in exp/lib_*.so; do
  GPUAGG_LIB=$PWD/$lib ABLATE_ONLY=${ABLATE_ONLY:-fwd,drop,c2} timeout -k 10 200 python scripts/ablate.py >> gpurun_out/exp_${TAG:-x}.jsonl 2>> gpurun_out/exp_${TAG:-x}.err || exit $?
done
