#!/bin/bash
# finalize1: bitonic order instead of O(n^2) ranks — hybrid parity tests, trace, configs[2] A/B
set -u
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_dropin_gpu.py tests/test_gpu_scan4.py tests/test_gpu_rerank.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
BB_SELECT_TRACE=1 timeout -k 10 120 python3 tools/scale_bench.py --cases c3 --seconds 0.2 > $O/c3d.jsonl 2> $O/c3d.err || exit 1
grep "finalize trace" $O/c3d.err | tail -1
for rep in 1 2; do for lib in new head; do
  if [ $lib = head ]; then L=BRICKREC_LIB=$(pwd)/tools/ab/libbrickrec_head.so; else L=X=1; fi
  timeout -k 10 200 env $L python3 bench.py --workload c3 --steps 300 --no-cpu > $O/c3_${lib}_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c3_${lib}_$rep.log').read().strip().splitlines()[-1]); print('c3 $lib', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
done; done
