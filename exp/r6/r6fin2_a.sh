#!/bin/bash
# round-6 final evidence, session A (final build: fold wait + balanced lanes + per-segment folds): every GPU test and the smoke at the tree's build
cd "$(dirname "$0")/../.."
bash scripts/gpu_check.sh r6fin2_a tests smoke
