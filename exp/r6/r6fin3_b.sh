#!/bin/bash
# session B: C2 (the driver's config) and C3 -- PMC passes first, so the bench lines carry traffic
cd "$(dirname "$0")/../.."
bash scripts/gpu_check.sh r6fin3_b pmc:c2 bench:c2 prof:c2 pprof:c2 pmc:c3 bench:c3 prof:c3
