#!/bin/bash
# round-6 final evidence, session A (final build: search-first hot-key cache): every GPU test and the smoke at the tree's build
cd "$(dirname "$0")/../.."
bash scripts/gpu_check.sh r6fin_a tests smoke
