#!/bin/bash
# index views (bb_create_view): GPU tests, then in-flight lanes as views vs own copies, 3 and 4 lanes
set -u
O=gpurun_out/r02v3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for args in "--inflight 3" "--inflight 4" "--inflight 5" "--inflight 3 --lane-copies"; do
    tag=$(echo $args | tr -d ' -')
    timeout -k 10 200 python3 bench.py --no-cpu --no-sweep $args > $O/b_${tag}_$rep.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$O/b_${tag}_$rep.log').read().strip().splitlines()[-1]); print('$args'.ljust(28), round(d['value']/1e6,3), d['p50_ms'], d['p50_ms_serial'], d['kernels_us_per_step'])"
  done
done
for args in "--inflight 3" "--inflight 3 --lane-copies"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 200 python3 bench.py --workload c3 --steps 300 --no-cpu $args > $O/c3_${tag}.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c3_${tag}.log').read().strip().splitlines()[-1]); print('c3 $args'.ljust(28), round(d['value']/1e6,3), d['p50_ms_serial'])"
done
