#!/bin/bash
# cheaper key hash (variant library): A/B vs the final build on c4-remote, c1, c5
cd "$(dirname "$0")/../.."
bash exp/r6/ab.sh r6z4_ab c4-remote exp/r6/lib_4afc.so exp/r6/lib_hash2.so || exit $?
bash exp/r6/ab.sh r6z4_ab1 c1 exp/r6/lib_4afc.so exp/r6/lib_hash2.so || exit $?
bash exp/r6/ab.sh r6z4_ab5 c5 exp/r6/lib_4afc.so exp/r6/lib_hash2.so
