#!/bin/bash
# Round-6 evidence on one box: smoke(), then per workload (configs[1] = c2, configs[2] = c3) the
# bench line with cpu_baseline, rocprofv3 --kernel-trace --stats of `bench.py --inflight 1`
# (warm) and of the same with the Infinity Cache flushed before every step (cold), and the
# FETCH_SIZE / WRITE_SIZE passes (tools/evidence_run.sh).  Output: gpurun_out/$1/.
set -u
T=${1:-r06fin}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -5 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
bash tools/evidence_run.sh $T ${2:-c2 c3}
