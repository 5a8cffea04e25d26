#!/bin/bash
# One parameterised GPU-box runner (replaces the per-round one-off scripts).
#
#   bash tools/gpu_run.sh TAG tests                     -m gpu parity tests
#   bash tools/gpu_run.sh TAG bench [ARGS] [-- ENV...]  bench.py line per env variant ("" = plain)
#   bash tools/gpu_run.sh TAG ablib [ARGS]              this tree's library vs tools/ab/libbrickrec_head.so, alternating
#   bash tools/gpu_run.sh TAG prof [ARGS]               rocprofv3 --kernel-trace --stats of bench.py ARGS
#   bash tools/gpu_run.sh TAG pmc [ARGS]                PMC passes (one counter group per run) of bench.py ARGS
#   bash tools/gpu_run.sh TAG traffic [ARGS]            the FETCH_SIZE and WRITE_SIZE passes only
#
# Several modes chain with "+": bash tools/gpu_run.sh r03a tests+bench+prof --workload c3
# Every GPU step runs under its own timeout; the first abnormal exit ends the script.
# Output: gpurun_out/TAG/ (copy what is judged into profiles/ with tools/collect_profiles.py).
set -u
T=$1; MODES=$2; shift 2
ARGS=(); ENVS=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; ENVS=("$@"); break; fi
  ARGS+=("$1"); shift
done
[ ${#ENVS[@]} -eq 0 ] && ENVS=("X=1")
R=$(pwd); O="$R/gpurun_out/$T"; mkdir -p "$O"

summ() {  # one bench JSON line -> short summary
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sw = [(s["B"], round(s["queries_per_s_inflight3"] / 1e6, 2), s["p50_ms_serial"]) for s in d.get("gpu_batch_sweep", [])]
print(sys.argv[2][:48].ljust(48), round(d["value"] / 1e6, 3), "M q/s", "serial", d.get("p50_ms_serial"),
      d.get("kernels_us_per_step"), "frac", d["roofline"]["frac"], sw)
EOF
}

for M in ${MODES//+/ }; do
  case $M in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
        > "$O/tests.log" 2>&1; rc=$?
      echo "tests rc=$rc"; tail -4 "$O/tests.log"; [ $rc -ne 0 ] && exit $rc ;;
    bench)
      i=0
      for e in "${ENVS[@]}"; do
        i=$((i+1))
        timeout -k 10 300 env BB_AB=1 $e python3 bench.py --no-cpu "${ARGS[@]}" > "$O/bench_$i.log" 2>&1; rc=$?
        [ $rc -ne 0 ] && { echo "bench[$e] rc=$rc"; tail -5 "$O/bench_$i.log"; exit $rc; }
        summ "$O/bench_$i.log" "$e"
      done ;;
    ablib)
      for rep in 1 2; do
        for lib in new head; do
          L=X=1; [ $lib = head ] && L=BRICKREC_LIB=$R/tools/ab/libbrickrec_head.so
          timeout -k 10 300 env $L python3 bench.py --no-cpu "${ARGS[@]}" > "$O/ab_${lib}_$rep.log" 2>&1; rc=$?
          [ $rc -ne 0 ] && { echo "ab $lib rc=$rc"; tail -3 "$O/ab_${lib}_$rep.log"; exit $rc; }
          summ "$O/ab_${lib}_$rep.log" "$lib"
        done
      done ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run \
          --output-format csv -- python3 "$R/bench.py" --no-cpu --no-sweep "${ARGS[@]}" > "$O/prof.log" 2>&1 ); rc=$?
      echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/prof.log"; exit $rc; }
      for f in $(find "$O/prof" -name "*kernel_stats.csv"); do head -12 "$f"; done ;;
    pmc|traffic)
      i=0
      PGROUPS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM"
              "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"
              "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT")
      [ $M = traffic ] && PGROUPS=("FETCH_SIZE" "WRITE_SIZE")   # HBM bytes only
      for grp in "${PGROUPS[@]}"; do
        i=$((i+1))
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$O/pmc/p$i" -o run \
            --output-format csv -- python3 "$R/bench.py" --steps 30 --warmup 5 --no-cpu --no-sweep --inflight 1 "${ARGS[@]}" \
            > "$O/pmc_p$i.log" 2>&1 ); rc=$?
        echo "pmc pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/pmc_p$i.log"; exit $rc; }
      done
      python3 "$R/tools/pmc_summary.py" "$O/pmc" > "$O/pmc_summary.json"; cat "$O/pmc_summary.json" ;;
    *) echo "unknown mode $M"; exit 2 ;;
  esac
done
exit 0
