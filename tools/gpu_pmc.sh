#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over a short bench.
set -u
R=$(pwd)
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/pmc/p$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 30 --warmup 5 --no-cpu --inflight 1 > "$R/gpurun_out/pmc/p$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/pmc/p$i.log"; exit $rc; }
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc" > "$R/gpurun_out/pmc/summary.json"
cat "$R/gpurun_out/pmc/summary.json"
