#!/bin/bash
# serial (one batch in flight) kernel trace of configs[1] and configs[2]: per-kernel durations and inter-kernel gaps
set -u
O=gpurun_out/r02t; mkdir -p $O
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-cpu --no-sweep --inflight 1 > "$R/$O/c2.log" 2>&1; rc=$?; echo "c2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/c3" -o run --output-format csv -- python3 "$R/bench.py" --workload c3 --steps 200 --warmup 20 --no-cpu --inflight 1 > "$R/$O/c3.log" 2>&1; rc=$?; echo "c3 rc=$rc"
exit $rc
