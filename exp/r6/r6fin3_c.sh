#!/bin/bash
# session C: C1, C4, C4 remote, C5
cd "$(dirname "$0")/../.."
bash scripts/gpu_check.sh r6fin3_c pmc:c1 bench:c1 prof:c1 pmc:c4 bench:c4 prof:c4 pmc:c4-remote bench:c4-remote prof:c4-remote pmc:c5 bench:c5 prof:c5 || exit $?
bash exp/r6/abflags.sh r6fin3_d c4-remote 0 512
