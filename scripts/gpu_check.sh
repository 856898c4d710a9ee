#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel-trace summary.
#   bash scripts/gpu_check.sh TAG [tests|bench|prof ...]   (default: all three)
# Every GPU step has its own time limit; a crash/timeout stops the script.
TAG=${1:-run}
shift
STEPS=${*:-tests bench prof}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
OUT="$R/gpurun_out"
mkdir -p "$OUT"
{ rocminfo | grep -m2 -E "Name: +gfx|Marketing Name: +AMD Instinct"; nproc; lscpu | grep "Model name"; } > "$OUT/${TAG}_info.txt" 2>&1
python -c "import __graft_entry__ as g; g.build()" > "$OUT/${TAG}_build.log" 2>&1 || exit 1
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -q -x > "$OUT/${TAG}_pytest.log" 2>&1
      rc=$?; echo "pytest rc=$rc" >> "$OUT/${TAG}_pytest.log"
      [ $rc -gt 1 ] && exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || exit $? ;;
    bench)
      timeout -k 10 600 python bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
      rc=$?; echo "bench rc=$rc" >> "$OUT/${TAG}_bench.err"; [ $rc -ne 0 ] && exit $rc ;;
    prof)
      export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run \
        -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/${TAG}_prof.log" 2>&1
      rc=$?; echo "prof rc=$rc" >> "$OUT/${TAG}_prof.log"; [ $rc -ne 0 ] && exit $rc ;;
  esac
done
exit 0
