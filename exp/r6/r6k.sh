#!/bin/bash
cd "$(dirname "$0")/../.."
bash exp/r6/ab.sh r6k_ab c3 tree exp/lib_skd21.so exp/lib_skd22.so
