#!/bin/bash
# Quick GPU check: all -m gpu tests, then the configs[1] bench line without the CPU leg,
# plus optional A/B env settings: bash tools/gpu_quick.sh TAG ["ENV=1 ..."]...
set -u
T=$1; shift
R=$(pwd); O="$R/gpurun_out/$T"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > "$O/gpu_all.log" 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 "$O/gpu_all.log"; [ $rc -ne 0 ] && exit $rc
i=0
for envs in "" "$@"; do
  i=$((i+1))
  timeout -k 10 200 env $envs python3 bench.py --no-cpu --steps 500 > "$O/bench_$i.log" 2>&1; rc=$?
  echo "bench[$envs] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/bench_$i.log"; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$i.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['p50_ms_serial'], d['kernels_us_per_step'], [ (s['B'], s['queries_per_s_inflight3'], s['p50_ms_serial']) for s in d.get('gpu_batch_sweep', [])])"
done
