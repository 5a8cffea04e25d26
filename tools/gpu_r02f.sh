#!/bin/bash
# Round-2 evidence of the current build: GPU suite (with the parity gate reports), smoke, then
# rocprofv3 stats + FETCH/WRITE PMC of configs[1..4] and the default bench line.
set -u
T=${1:-r02f}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread > $O/gpu_all.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/gpu_all.log; grep "\[parity\]" $O/gpu_all.log | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_prof_r02.sh $T c2 c3 c4 c5
