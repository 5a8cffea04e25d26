#!/bin/bash
# A/B of env-selected variants: bench line (per-kernel event times) + rocprofv3 stats each.
set -u
R=$(pwd); O="$R/gpurun_out/ab"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for v in "${@}"; do
  i=$((i+1))
  env $v timeout -k 10 300 python3 "$R/bench.py" --steps 300 --warmup 30 --no-cpu > "$O/b$i.log" 2>&1; rc=$?
  echo "[$v] rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$O/b$i.log") $(grep -o '"kernels_us_per_step": {[^}]*}' "$O/b$i.log")"
  [ $rc -ne 0 ] && { tail -5 "$O/b$i.log"; exit $rc; }
done
exit 0
