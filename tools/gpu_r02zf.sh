#!/bin/bash
# final evidence: GPU suite, smoke, default bench line, configs[2] line, rocprofv3 stats of both
set -u
O=gpurun_out/r02zf; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread > $O/gpu_all.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" $O/gpu_all.log | tail -1; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 bench.py --workload c3 --steps 500 --no-cpu > $O/bench_c3.log 2>&1; rc=$?; echo "bench c3 rc=$rc"; [ $rc -ne 0 ] && exit $rc
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-cpu --no-sweep > "$R/$O/prof_c2.log" 2>&1; rc=$?; echo "prof c2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_c3" -o run --output-format csv -- python3 "$R/bench.py" --workload c3 --steps 200 --warmup 20 --no-cpu > "$R/$O/prof_c3.log" 2>&1; rc=$?; echo "prof c3 rc=$rc"
exit $rc
