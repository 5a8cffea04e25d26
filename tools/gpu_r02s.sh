#!/bin/bash
# DPP f64 wave sums in prep / row conversion: GPU suite, then A/B vs the head library (configs[1], configs[2])
set -u
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for lib in new head; do
  if [ $lib = head ]; then L=BRICKREC_LIB=$(pwd)/tools/ab/libbrickrec_head.so; else L=X=1; fi
  timeout -k 10 200 env $L python3 bench.py --no-cpu --no-sweep > $O/c2_${lib}_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c2_${lib}_$rep.log').read().strip().splitlines()[-1]); print('c2 $lib', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
  timeout -k 10 200 env $L python3 bench.py --workload c3 --steps 300 --no-cpu > $O/c3_${lib}_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c3_${lib}_$rep.log').read().strip().splitlines()[-1]); print('c3 $lib', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
done; done
