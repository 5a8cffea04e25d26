#!/bin/bash
# blocked scan2 image + int16 re-rank image: full GPU suite, then A/B of BB_S16 modes vs head lib
set -u
O=gpurun_out/r02u; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r02u_ab "BB_S16=2" "BB_S16=0" "HEAD" || exit 1
for e in X=1 BB_S16=2 BB_S16=0; do
  timeout -k 10 200 env $e python3 bench.py --workload c3 --steps 300 --no-cpu > $O/c3_$e.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c3_$e.log').read().strip().splitlines()[-1]); print('c3 $e', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
done
