#!/bin/bash
# Diagnostic builds of the engine library with -D experiment switches (not product code).
# A variant "A+B" defines both A and B; "" is the unmodified build.
cd "$(dirname "$0")/.."
rm -f exp/lib_*.so
for v in "$@"; do
  name=${v:-base}
  python retina_amd/build.py --variant exp/lib_$name.so ${v//+/ } > /tmp/bv_$name.log 2>&1 &
done
wait
ls -la exp/*.so
