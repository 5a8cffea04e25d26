#!/bin/bash
# query-block-major tile maxima: GPU suite, configs[1] A/B vs previous library, c3, c4 shard sweep line
set -u
O=gpurun_out/r02zc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r02zc_ab "HEAD" || exit 1
for f in $O/../r02zc_ab/ab_*_1.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['kernels_us_per_step'])"; done
timeout -k 10 200 python3 bench.py --workload c3 --steps 300 --no-cpu > $O/c3.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/c3.log').read().strip().splitlines()[-1]); print('c3', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
for lib in new head; do
  if [ $lib = head ]; then L=BRICKREC_LIB=$(pwd)/tools/ab/libbrickrec_head.so; else L=X=1; fi
  timeout -k 10 300 env $L python3 tools/scale_bench.py --cases c4-shard --seconds 1 > $O/c4s_$lib.jsonl 2> $O/c4s_$lib.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/c4s_$lib.jsonl').read().strip().splitlines()[-1]); print('c4-shard $lib', d['ms_per_batch'], d['kernels_us_per_batch'], d.get('frac_end_to_end'))"
done
