#!/bin/bash
# MFMA probe, counter list, rocprofv3 kernel-trace/stats of a short bench run.
set -u
R=$(pwd)
mkdir -p "$R/gpurun_out/prof"
timeout -k 10 120 ./tools/mfma_probe > gpurun_out/mfma_probe.jsonl 2>&1; rc=$?
echo "probe rc=$rc"; cat gpurun_out/mfma_probe.jsonl
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-cpu > "$R/gpurun_out/prof_bench.log" 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -3 "$R/gpurun_out/prof_bench.log"
find "$R/gpurun_out/prof" -name "*stats*" | head; 
for f in $(find "$R/gpurun_out/prof" -name "*kernel_stats.csv"); do cat "$f"; done
exit $rc
