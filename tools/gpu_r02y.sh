#!/bin/bash
# scan2 with two workgroups per CU (BB_SCAN_OCC2=1): re-rank tests under it, A/B
set -u
O=gpurun_out/r02y; mkdir -p $O
BB_SCAN_OCC2=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_rerank.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r02y_ab "BB_SCAN_OCC2=1" || exit 1
for f in $O/../r02y_ab/ab_*_1.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['kernels_us_per_step'])"; done
