#!/bin/bash
# round-6 final evidence, session A (final build: + 32-byte list entries by default): every GPU test and the smoke at the tree's build
cd "$(dirname "$0")/../.."
bash scripts/gpu_check.sh r6fin3_a tests smoke
