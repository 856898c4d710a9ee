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
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
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
    micro)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/mb scripts/microbench.hip > "$OUT/${TAG}_micro.err" 2>&1 || exit 1
      timeout -k 10 300 /tmp/mb > "$OUT/${TAG}_micro.jsonl" 2>> "$OUT/${TAG}_micro.err"
      rc=$?; echo "micro rc=$rc" >> "$OUT/${TAG}_micro.err"; [ $rc -ne 0 ] && exit $rc ;;
    microlds)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/mbl scripts/microbench_lds.hip > "$OUT/${TAG}_microlds.err" 2>&1 || exit 1
      timeout -k 10 300 /tmp/mbl > "$OUT/${TAG}_microlds.jsonl" 2>> "$OUT/${TAG}_microlds.err"
      rc=$?; echo "microlds rc=$rc" >> "$OUT/${TAG}_microlds.err"; [ $rc -ne 0 ] && exit $rc ;;
    ablate)
      timeout -k 10 600 python scripts/ablate.py > "$OUT/${TAG}_ablate.jsonl" 2> "$OUT/${TAG}_ablate.err"
      rc=$?; echo "ablate rc=$rc" >> "$OUT/${TAG}_ablate.err"; [ $rc -ne 0 ] && exit $rc ;;
    pmc)
      # one counter group per pass (MI355X_MICROARCH.md: rocprofv3 PMC slots)
      export TMPDIR=/tmp
      rocprofv3 -L > "$OUT/${TAG}_counters.txt" 2>&1
      i=0
      for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
                 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT GRBM_GUI_ACTIVE" \
                 "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
        i=$((i+1))
        timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/${TAG}_pmc$i" -o run \
          -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline \
          > "$OUT/${TAG}_pmc$i.log" 2>&1
        rc=$?; echo "pmc$i rc=$rc" >> "$OUT/${TAG}_pmc$i.log"
        [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
      done
      python scripts/pmc_summary.py "$OUT/${TAG}_pmc_c2.json" dense_ 100000000 "$OUT/${TAG}_pmc4" "$OUT/${TAG}_pmc5" \
        > /dev/null 2>> "$OUT/${TAG}_pmc5.log" ;;
  esac
done
exit 0
