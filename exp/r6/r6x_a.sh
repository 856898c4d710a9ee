#!/bin/bash
# round-6 final evidence, session A (build after the wide-key fold changes): every GPU test and the smoke at the tree's build
cd "$(dirname "$0")/../.."
bash scripts/gpu_check.sh r6xa tests smoke
