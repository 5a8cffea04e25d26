#!/bin/bash
# scan2: first tiles' DMA issued before the query loads; GPU suite + configs[1] A/B vs head
set -u
O=gpurun_out/r02l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r02l_ab "HEAD" || exit 1
for f in $O/../r02l_ab/ab_*_1.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['kernels_us_per_step'])"; done
