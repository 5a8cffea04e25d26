#!/bin/bash
# scan5 (16x16x32 streaming scan, d = 768): streaming + configs GPU tests, then c4 A/B vs BB_SCAN5=0
set -u
O=gpurun_out/r02h5; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_configs.py tests/test_gpu_scan4.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -25; [ $rc -ne 0 ] && exit $rc
for e in X=1 BB_SCAN5=0; do
  timeout -k 10 300 env $e python3 tools/scale_bench.py --cases c4-shard,c4-full,c4-B1024 --seconds 1 > $O/c4_$e.jsonl 2> $O/c4_$e.err || { tail -5 $O/c4_$e.err; exit 1; }
  python3 -c "
import json
for l in open('$O/c4_$e.jsonl'):
    d=json.loads(l); print('$e', d['case'], d['ms_per_batch'], d['kernels_us_per_batch'], d.get('frac_end_to_end'))"
done
