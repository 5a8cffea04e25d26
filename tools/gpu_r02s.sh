#!/bin/bash
# XCD row mapping + fat wave rescore: re-rank GPU tests, then A/B vs the head library
set -u
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rerank.py tests/test_gpu_configs.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_lib.sh r02s || exit 1
bash tools/gpu_ab_lib.sh r02s3 --workload c3 --steps 300
