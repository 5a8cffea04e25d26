#!/bin/bash
# A/B of env settings (and the head library) on one box, configs[1] bench line without the CPU
# leg, two alternations: bash tools/gpu_ab_env.sh TAG "ENV=1 ..." ... (HEAD = tools/ab library)
set -u
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  i=0
  for envs in "X=1" "$@"; do
    i=$((i+1))
    e=${envs/HEAD/BRICKREC_LIB=$(pwd)/tools/ab/libbrickrec_head.so}
    timeout -k 10 200 env $e python3 bench.py --no-cpu > $O/ab_${i}_$rep.log 2>&1 || { tail -3 $O/ab_${i}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/ab_${i}_$rep.log').read().strip().splitlines()[-1]); print('$envs'[:40].ljust(40), round(d['value']/1e6,3), 'M q/s', d['p50_ms_serial'], [ (s['B'], round(s['queries_per_s_inflight3']/1e6,2), s['p50_ms_serial']) for s in d.get('gpu_batch_sweep', [])])"
  done
done
