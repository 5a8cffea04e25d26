#!/bin/bash
# consolidated sweep of this build (serial + 3 in flight) and the configs[1] line at 2/4/6 batches in flight
set -u
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 900 python3 tools/scale_bench.py --cases c2-B1,c2-B256,c2-B1024,c2-B4096,c3,c4-shard,c4-full,c5-shard,c5-full,c4-B1,c4-B256,c4-B1024,f32-1M --seconds 1 --inflight 3 --out $O/sweep.jsonl > $O/sweep.log 2>&1; rc=$?
echo "sweep rc=$rc"; tail -3 $O/sweep.log; [ $rc -ne 0 ] && exit $rc
for n in 2 4 6; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-sweep --inflight $n > $O/inflight_$n.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/inflight_$n.log').read().strip().splitlines()[-1]); print('inflight $n', round(d['value']/1e6,3), d['p50_ms'], d['p50_ms_serial'])"
done
