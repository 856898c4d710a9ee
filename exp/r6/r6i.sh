#!/bin/bash
cd "$(dirname "$0")/../.."
bash exp/r6/ab.sh r6i_ab c2 tree exp/lib_nostore.so exp/lib_noqflush.so exp/lib_nospill.so
