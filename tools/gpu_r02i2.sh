#!/bin/bash
# one-row-per-workgroup prep + fatter re-rank rescore: re-rank / parity tests, configs[1] A/B, in-flight depth
set -u
O=gpurun_out/r02i2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rerank.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r02i2_ab "BB_PREP_ROWS=4" "HEAD" || exit 1
for f in $O/../r02i2_ab/ab_*_1.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['kernels_us_per_step'])"; done
for n in 3 4 3 4; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-sweep --inflight $n > $O/inflight_$n.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/inflight_$n.log').read().strip().splitlines()[-1]); print('inflight $n', round(d['value']/1e6,3), d['p50_ms'], d['p50_ms_serial'])"
done
