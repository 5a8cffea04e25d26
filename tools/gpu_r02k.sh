#!/bin/bash
# final evidence of the round: GPU suite (parity gate reports), smoke, bench line, rocprofv3 stats of the bench command
set -u
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread > $O/gpu_all.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" $O/gpu_all.log | tail -1; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-cpu --no-sweep > "$R/$O/prof_c2.log" 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
