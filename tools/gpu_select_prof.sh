#!/bin/bash
# rocprofv3 kernel durations of the select kernel under each BB_SELECT_ABLATE variant
# (serial bench, one in-flight batch).  Each GPU step has its own limit; stop at the first failure.
set -u
R=$(pwd)
rm -rf "$R/gpurun_out/sprof"; mkdir -p "$R/gpurun_out/sprof"
cd /tmp && export TMPDIR=/tmp
for a in ${ABLS:-0 1 2 4}; do
  BB_SELECT_ABLATE=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/sprof/a$a" -o run --output-format csv -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-cpu --inflight 1 ${BENCH_ARGS:-} > "$R/gpurun_out/sprof/a$a.log" 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "abl=$a rc=$rc"; tail -5 "$R/gpurun_out/sprof/a$a.log"; exit $rc; }
  f=$(find "$R/gpurun_out/sprof/a$a" -name "*kernel_stats.csv" | head -1)
  echo "abl=$a $(grep -E 'select_kernel|scan3_kernel|prep_kernel' "$f" | awk -F'","' '{split($1,n,"("); printf "%s=%s ", substr(n[1],2), $4}')"
done
