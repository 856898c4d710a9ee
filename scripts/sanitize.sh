#!/bin/bash
# Host-sanitizer runs of the library's C++ side over the whole CPU test files (CPU box; no GPU).
#   bash scripts/sanitize.sh [asan|tsan ...]      (default: both)
# Builds /tmp/gpuagg_<kind>/libgpuagg_<kind>.so (retina_amd/build.py build_sanitized), preloads
# the clang runtime into python and points GPUAGG_LIB at it.  Reports go to /tmp/gpuagg_<kind>/report.*;
# the script fails if any report was written or a test failed.  tests/test_sanitize.py runs a selection.
cd "$(dirname "$0")/.." || exit 1
KINDS=${*:-asan tsan}
rc=0
for kind in $KINDS; do
  lib=$(python retina_amd/build.py --sanitize "$kind") || exit 1
  rt=$(/opt/rocm/bin/hipcc -print-file-name="libclang_rt.${kind}-x86_64.so")
  dir=$(dirname "$lib")
  rm -f "$dir"/report.*
  files="tests/test_cpu_shard.py tests/test_cpu_backend.py"
  [ "$kind" = asan ] && files="tests/test_cpu_abi.py $files"
  LD_PRELOAD=$rt GPUAGG_LIB=$lib \
    ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:log_path=$dir/report" \
    UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:log_path=$dir/report" \
    TSAN_OPTIONS="report_signal_unsafe=0:halt_on_error=0:log_path=$dir/report" \
    python -m pytest -q -p no:cacheprovider -m "not gpu" $files
  r=$?
  if ls "$dir"/report.* > /dev/null 2>&1; then
    echo "$kind: reports in $dir:"; ls "$dir"/report.*; r=1
  fi
  echo "$kind: rc=$r"
  [ $r -ne 0 ] && rc=$r
done
exit $rc
