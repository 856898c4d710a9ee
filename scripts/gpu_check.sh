#!/bin/bash
# One GPU-box session: parity tests, bench lines, rocprofv3 summaries, PMC passes.
#   bash scripts/gpu_check.sh TAG STEP...
# STEP: build | tests[:PYTEST_ARGS] | smoke | bench:CFG | prof:CFG | pprof:CFG | pmc:CFG | micro | microlds
#       (CFG = c1..c5, default c2; tests:k=A,B runs `-k "A or B"`)
# Every GPU step has its own time limit; a crash, abort or timeout stops the script.
TAG=${1:-run}
shift
STEPS=${*:-tests bench:c2 prof:c2}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
OUT="$R/gpurun_out"
mkdir -p "$OUT"
{ rocminfo | grep -m2 -E "Name: +gfx|Marketing Name: +AMD Instinct"; nproc; lscpu | grep "Model name"; } > "$OUT/${TAG}_info.txt" 2>&1
export TMPDIR=/tmp
# generated workloads are cached across this session's bench / prof / pmc runs (bench.py)
export BENCH_CACHE=/tmp/benchcache_$TAG
for s in $STEPS; do
  name=${s%%:*}
  arg=""
  [ "$name" != "$s" ] && arg=${s#*:}
  cfg=${arg:-c2}
  echo "$(date +%T) step $s" >> "$OUT/${TAG}_steps.txt"
  case $name in
    build)
      python -c "import __graft_entry__ as g; g.build()" > "$OUT/${TAG}_build.log" 2>&1 || exit 1 ;;
    tests)
      sel=()
      # k=a,b,c selects tests matching any of a, b, c (steps are split on whitespace)
      [ -n "$arg" ] && { k=${arg#k=}; sel=(-k "${k//,/ or }"); }
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${sel[@]}" \
        > "$OUT/${TAG}_pytest.log" 2>&1
      rc=$?; echo "pytest rc=$rc" >> "$OUT/${TAG}_pytest.log"
      [ $rc -ne 0 ] && exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || exit $? ;;
    bench)
      timeout -k 10 600 python bench.py --config "$cfg" > "$OUT/${TAG}_bench_${cfg}.json" 2> "$OUT/${TAG}_bench_${cfg}.err"
      rc=$?; echo "bench rc=$rc" >> "$OUT/${TAG}_bench_${cfg}.err"; [ $rc -ne 0 ] && exit $rc ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_${cfg}" -o run \
        -- python3 "$R/bench.py" --config "$cfg" --steps 5 --warmup 1 --no-cpu-baseline --no-host-fed --no-production --no-scrape \
        > "$OUT/${TAG}_prof_${cfg}.log" 2>&1
      rc=$?; echo "prof rc=$rc" >> "$OUT/${TAG}_prof_${cfg}.log"; [ $rc -ne 0 ] && exit $rc
      find "$OUT/${TAG}_prof_${cfg}" -name "*kernel_stats.csv" -exec cp {} "$OUT/${TAG}_${cfg}_kernel_stats.csv" \; ;;
    pprof)
      # the production-geometry launches alone (bench.py --production-only)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_pprof_${cfg}" -o run \
        -- python3 "$R/bench.py" --config "$cfg" --production-only > "$OUT/${TAG}_pprof_${cfg}.log" 2>&1
      rc=$?; echo "pprof rc=$rc" >> "$OUT/${TAG}_pprof_${cfg}.log"; [ $rc -ne 0 ] && exit $rc
      find "$OUT/${TAG}_pprof_${cfg}" -name "*kernel_stats.csv" -exec cp {} "$OUT/${TAG}_${cfg}_pprof_kernel_stats.csv" \; ;;
    pmc)
      # one counter group per pass (MI355X_MICROARCH.md: rocprofv3 PMC slots; TCC: FETCH_SIZE
      # uses 3 of 4, WRITE_SIZE 2, so they take separate passes)
      i=0
      for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
                 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_INSTS_LDS_ATOMIC GRBM_GUI_ACTIVE" \
                 "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum"; do
        i=$((i+1))
        timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/${TAG}_pmc_${cfg}_$i" -o run \
          -- python3 "$R/bench.py" --config "$cfg" --steps 2 --warmup 1 --no-cpu-baseline --no-host-fed --no-production --no-scrape \
          > "$OUT/${TAG}_pmc_${cfg}_$i.log" 2>&1
        rc=$?; echo "pmc$i rc=$rc" >> "$OUT/${TAG}_pmc_${cfg}_$i.log"
        [ $rc -ne 0 ] && exit $rc
      done
      python scripts/pmc_summary.py "$OUT/${TAG}_pmc_${cfg}.json" "$(python scripts/bench_field.py "$OUT/${TAG}_pmc_${cfg}_1.log" roofline.kernel)" \
        "$(python scripts/bench_field.py "$OUT/${TAG}_pmc_${cfg}_1.log" config.records_per_gpu)" \
        "$(python scripts/bench_field.py "$OUT/${TAG}_pmc_${cfg}_1.log" build_id)" "$OUT"/${TAG}_pmc_${cfg}_[0-9]* > /dev/null 2>> "$OUT/${TAG}_pmc_${cfg}_1.log"
      # this box's later bench lines read the fresh summary (bench.py takes it only when its
      # build id is the loaded library's); scripts/collect_round.py copies it into the tree
      [ -s "$OUT/${TAG}_pmc_${cfg}.json" ] && cp "$OUT/${TAG}_pmc_${cfg}.json" "$R/profiles/pmc_${cfg}.json" ;;
    ablate)
      ABLATE_ONLY="$arg" timeout -k 10 600 python scripts/ablate.py > "$OUT/${TAG}_ablate.jsonl" 2> "$OUT/${TAG}_ablate.err"
      rc=$?; echo "ablate rc=$rc" >> "$OUT/${TAG}_ablate.err"; [ $rc -ne 0 ] && exit $rc ;;
    micro)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/mb scripts/microbench.hip > "$OUT/${TAG}_micro.err" 2>&1 || exit 1
      timeout -k 10 300 /tmp/mb > "$OUT/${TAG}_micro.jsonl" 2>> "$OUT/${TAG}_micro.err"
      rc=$?; echo "micro rc=$rc" >> "$OUT/${TAG}_micro.err"; [ $rc -ne 0 ] && exit $rc ;;
    microlds)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/mbl scripts/microbench_lds.hip > "$OUT/${TAG}_microlds.err" 2>&1 || exit 1
      timeout -k 10 300 /tmp/mbl > "$OUT/${TAG}_microlds.jsonl" 2>> "$OUT/${TAG}_microlds.err"
      rc=$?; echo "microlds rc=$rc" >> "$OUT/${TAG}_microlds.err"; [ $rc -ne 0 ] && exit $rc ;;
    *)
      echo "unknown step $s" >> "$OUT/${TAG}_steps.txt"; exit 2 ;;
  esac
done
exit 0
