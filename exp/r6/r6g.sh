#!/bin/bash
cd "$(dirname "$0")/../.."
bash exp/r6/ab.sh r6g_ab c2 tree exp/lib_ntspill.so
