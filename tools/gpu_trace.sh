#!/bin/bash
# Select-phase traces (serial configs[1]); extra args: env settings per run
set -u
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
i=0
for envs in "" "$@"; do
  i=$((i+1))
  timeout -k 10 120 env BB_SELECT_TRACE=1 $envs python3 bench.py --no-cpu --no-sweep --inflight 1 --steps 10 --warmup 2 > $O/trace_$i.log 2>&1 || exit $?
  echo "[$envs]"; grep "wave select trace" $O/trace_$i.log | tail -1
done
