#!/bin/bash
cd "$(dirname "$0")/../.."
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 ./scripts/mbl > $OUT/r6e_mbl.jsonl 2> $OUT/r6e_mbl.err || exit $?
bash exp/r6/ab.sh r6e_ab c2 tree exp/lib_nospill.so exp/lib_noflush.so exp/lib_noatomic.so exp/lib_nolookup.so
