#!/bin/bash
# finalize1: both sides' lists and the rank-0 key loaded in one round: GPU suite, trace, A/B vs head
set -u
O=gpurun_out/r02zj; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for lib in new head; do
  if [ $lib = head ]; then L=BRICKREC_LIB=$(pwd)/tools/ab/libbrickrec_head.so; else L=X=1; fi
  BB_SELECT_TRACE=1 timeout -k 10 120 env $L python3 tools/scale_bench.py --cases c3 --seconds 0.2 > $O/c3d_$lib.jsonl 2> $O/c3d_$lib.err || exit 1
  echo "$lib: $(grep 'finalize trace' $O/c3d_$lib.err | tail -1)"
done
for rep in 1 2; do for lib in new head; do
  if [ $lib = head ]; then L=BRICKREC_LIB=$(pwd)/tools/ab/libbrickrec_head.so; else L=X=1; fi
  timeout -k 10 200 env $L python3 bench.py --no-cpu --no-sweep > $O/c2_${lib}_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c2_${lib}_$rep.log').read().strip().splitlines()[-1]); print('c2 $lib', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
  timeout -k 10 200 env $L python3 bench.py --workload c3 --steps 300 --no-cpu > $O/c3_${lib}_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c3_${lib}_$rep.log').read().strip().splitlines()[-1]); print('c3 $lib', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
done; done
