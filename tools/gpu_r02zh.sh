#!/bin/bash
# probe: prep launched twice per step (BB_PREP_TWICE) — the second launch runs with warm
# instruction / data caches; serial kernel trace of configs[1]
set -u
O=gpurun_out/r02zh; mkdir -p $O
R=$(pwd); cd /tmp && export TMPDIR=/tmp
BB_PREP_TWICE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/$O/c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 10 --no-cpu --no-sweep --inflight 1 > "$R/$O/c2.log" 2>&1; rc=$?; echo "c2 rc=$rc"
exit $rc
