#!/bin/bash
# A/B timings on one GPU box: scripts/ablate.py against the product library and each
# experiment library (exp/variant.py builds), same process layout, one JSON line per run.
#   bash scripts/ab.sh TAG ONLY LIB...   (LIB "base" = retina_amd/libgpuagg.so)
TAG=$1; ONLY=$2; shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    path=""
    [ "$lib" != "base" ] && path="$PWD/$lib"
    GPUAGG_LIB=$path ABLATE_ONLY=$ONLY timeout -k 10 300 python scripts/ablate.py \
      >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err
    rc=$?; echo "$lib rep $rep rc=$rc" >> gpurun_out/${TAG}_ab.err
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
