#!/bin/bash
# sparse_fold_wide_kernel cost breakdown (c4-remote): inserts / list reads / segment load+store
cd "$(dirname "$0")/../.."
bash exp/r6/ab.sh r6o_ab c4-remote tree exp/r6/lib_f_noins.so exp/r6/lib_f_nolist.so exp/r6/lib_f_noseg.so
