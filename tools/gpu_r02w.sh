#!/bin/bash
# wave-select gather (ballot compaction, one round) : rerank tests, traces, A/B
set -u
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rerank.py tests/test_gpu_configs.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for c in c2-B1024 c3; do
  BB_SELECT_TRACE=1 timeout -k 10 120 python3 tools/scale_bench.py --cases $c --seconds 0.2 > $O/$c.jsonl 2> $O/$c.err; rc=$?
  echo "$c rc=$rc"; grep "wave select trace" $O/$c.err | tail -2; [ $rc -ne 0 ] && { tail -5 $O/$c.err; exit $rc; }
done
timeout -k 10 200 python3 bench.py --workload c3 --steps 300 --no-cpu > $O/c3.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/c3.log').read().strip().splitlines()[-1]); print('c3', round(d['value']/1e6,3), d['p50_ms_serial'], d['kernels_us_per_step'])"
