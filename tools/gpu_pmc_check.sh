#!/bin/bash
# PMC passes over tools/scan3_check (per-variant scan3 and select kernels), kernel-trace only.
# Counter groups: PMC_GROUPS (";"-separated), default = issue/wait breakdown + instruction mix.
set -u
R=$(pwd)
rm -rf "$R/gpurun_out/pmc3"; mkdir -p "$R/gpurun_out/pmc3"
cd /tmp && export TMPDIR=/tmp
GROUPS_DEFAULT="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM;SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/pmc3/p$i" -o run --output-format csv -- "$R/tools/scan3_check" > "$R/gpurun_out/pmc3/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/pmc3/p$i.log"; exit $rc; }
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc3" > "$R/gpurun_out/pmc3/summary.json"
