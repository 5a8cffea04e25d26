#!/bin/bash
# Re-entry check: GPU tests, smoke, default bench line, rocprofv3 kernel stats of the bench command.
set -u
T=${1:-r02p}
R=$(pwd); O="$R/gpurun_out/$T"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$O/gpu_all.log" 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 "$O/gpu_all.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py > "$O/bench.log" 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 "$O/bench.log"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-cpu --no-sweep > "$O/prof_c2.log" 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
