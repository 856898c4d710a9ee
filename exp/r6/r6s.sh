#!/bin/bash
# wide-list fold threshold (cap/2 vs 3/4 vs 7/8), c4-remote and c1
cd "$(dirname "$0")/../.."
bash exp/r6/ab.sh r6s_ab c4-remote tree exp/r6/lib_thr34.so exp/r6/lib_thr78.so || exit $?
bash exp/r6/ab.sh r6s_ab1 c1 tree exp/r6/lib_thr34.so exp/r6/lib_thr78.so
