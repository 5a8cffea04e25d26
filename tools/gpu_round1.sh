#!/bin/bash
# Round evidence on one MI355X: parity tests, the bench line, a rocprofv3 kernel-trace/stats
# profile of the same bench command, and the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE).
# Every GPU step has its own time limit; the script stops at the first abnormal exit.
set -u
R=$(pwd)
O="$R/gpurun_out/${TAG:-r01}"
mkdir -p "$O/prof" "$O/pmc"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 "$O/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/bench.log" 2>&1; rc=$?
echo "bench rc=$rc"; tail -2 "$O/bench.log"
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o bench --output-format csv -- python3 "$R/bench.py" --no-cpu --inflight 1 ${BENCH_ARGS:-} > "$O/prof_bench.log" 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -1 "$O/prof_bench.log"
[ $rc -ne 0 ] && exit $rc
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$O/pmc/p$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 30 --warmup 5 --no-cpu --inflight 1 ${BENCH_ARGS:-} > "$O/pmc/p$i.log" 2>&1; rc=$?
  echo "pmc $grp rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$O/pmc/p$i.log"; exit $rc; }
done
python3 "$R/tools/pmc_summary.py" "$O/pmc" > "$O/pmc/summary.json"
for f in $(find "$O/prof" -name "*kernel_stats.csv"); do cat "$f"; done
