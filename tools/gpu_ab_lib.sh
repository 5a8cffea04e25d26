#!/bin/bash
# A/B of two library builds on one box: this tree's libbrickrec.so vs tools/ab/libbrickrec_head.so,
# alternating, configs[1] bench line (no CPU leg); extra args go to bench.py.
set -u
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  for lib in new head; do
    if [ $lib = head ]; then L=BRICKREC_LIB=$(pwd)/tools/ab/libbrickrec_head.so; else L=X=1; fi
    timeout -k 10 200 env $L python3 bench.py --no-cpu "$@" > $O/ab_${lib}_$rep.log 2>&1 || { tail -3 $O/ab_${lib}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/ab_${lib}_$rep.log').read().strip().splitlines()[-1]); print('$lib', round(d['value']/1e6,3), 'M q/s', d['p50_ms_serial'], [ (s['B'], round(s['queries_per_s_inflight3']/1e6,2), s['p50_ms_serial']) for s in d.get('gpu_batch_sweep', [])])"
  done
done
