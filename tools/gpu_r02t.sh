#!/bin/bash
# int16 score image on the re-rank path: GPU parity tests, then A/B (S16 default vs BB_S16=0 vs head lib)
set -u
O=gpurun_out/r02t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rerank.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_dropin_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r02t_ab "BB_S16=0" "HEAD" || exit 1
for e in X=1 BB_S16=0; do
  timeout -k 10 200 env $e python3 bench.py --workload c3 --steps 300 --no-cpu > $O/c3_$e.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c3_$e.log').read().strip().splitlines()[-1]); print('c3 $e', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
done
