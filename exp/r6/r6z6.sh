#!/bin/bash
# entry size at build 1b7915e3 (balanced, per-segment folds): C1 and c4-remote
cd "$(dirname "$0")/../.."
bash exp/r6/abflags.sh r6z6_ab1 c1 0 512
