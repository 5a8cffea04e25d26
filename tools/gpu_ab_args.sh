#!/bin/bash
# A/B of bench.py argument sets: one bench line each (no CPU baseline).
set -u
R=$(pwd); O="$R/gpurun_out/ab"; mkdir -p "$O"
i=0
for v in "${@}"; do
  i=$((i+1))
  timeout -k 10 300 python3 "$R/bench.py" --steps 500 --warmup 50 --no-cpu $v > "$O/a$i.log" 2>&1; rc=$?
  echo "[$v] rc=$rc $(grep -o '"value": [0-9.]*' "$O/a$i.log") $(grep -o '"ms_per_step": [0-9.]*' "$O/a$i.log") $(grep -o '"p50_ms": [0-9.]*' "$O/a$i.log") $(grep -o '"kernels_us_per_step": {[^}]*}' "$O/a$i.log")"
  [ $rc -ne 0 ] && { tail -5 "$O/a$i.log"; exit $rc; }
done
exit 0
