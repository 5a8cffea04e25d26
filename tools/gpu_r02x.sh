#!/bin/bash
# paired-halves blocked image: full GPU suite, A/B vs the session-start library, configs[2]
set -u
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r02x_ab "HEAD" || exit 1
timeout -k 10 200 python3 bench.py --workload c3 --steps 300 --no-cpu > $O/c3.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/c3.log').read().strip().splitlines()[-1]); print('c3', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
for f in $O/../r02x_ab/ab_*_1.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['kernels_us_per_step'])"; done
