#!/bin/bash
# strided fallback select: GPU suite, configs[2] A/B (dual vs not), configs[1] line vs the previous library
set -u
O=gpurun_out/r02zb; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for e in X=1 BB_DUAL=0; do
  timeout -k 10 200 env $e python3 bench.py --workload c3 --steps 300 --no-cpu > $O/c3_${e}_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c3_${e}_$rep.log').read().strip().splitlines()[-1]); print('c3 $e', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
done; done
bash tools/gpu_ab_env.sh r02zb_ab "HEAD"
