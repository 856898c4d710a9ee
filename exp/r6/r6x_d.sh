#!/bin/bash
# 24- vs 32-byte wide-list entries (FLAG_WIDE_ENTRIES = 512) at the evidence build; PMC of the 32-byte form
cd "$(dirname "$0")/../.."
bash exp/r6/abflags.sh r6xd_ab c4-remote 0 512 || exit $?
bash exp/r6/abflags.sh r6xd_ab1 c1 0 512 || exit $?
GPUAGG_BENCH_FLAGS=512 bash scripts/gpu_check.sh r6xd pmc:c4-remote
