#!/bin/bash
# round 5 probes: C5 without IP-table gathers (upper bound), C2 with full-size deferred folds
cd "$(dirname "$0")/.."
O=gpurun_out/r5f
for lib in "" exp/lib_c5ng.so; do
  GPUAGG_LIB=${lib:+$PWD/$lib} ABLATE_N=1000000 ABLATE_ONLY=c5,c5-retrans,c5-flags,c5-dns \
    timeout -k 10 240 python scripts/ablate.py >> ${O}_c5.jsonl 2>> ${O}.err || exit $?
done
for lib in "" exp/lib_c2defer.so; do
  GPUAGG_LIB=${lib:+$PWD/$lib} ABLATE_ONLY=c2,c4-zipf timeout -k 10 300 python scripts/ablate.py >> ${O}_c2.jsonl 2>> ${O}.err || exit $?
done
