#!/bin/bash
# hardware-queue count vs in-flight depth at configs[1] (bench line without the CPU leg)
set -u
O=gpurun_out/r02r; mkdir -p $O
for q in 4 8 16; do for L in 3 4 6 8; do
  [ $q = 4 ] && [ $L -gt 4 ] && continue
  timeout -k 10 200 env GPU_MAX_HW_QUEUES=$q python3 bench.py --no-cpu --no-sweep --inflight $L > $O/q${q}_l$L.log 2>&1 || { tail -3 $O/q${q}_l$L.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/q${q}_l$L.log').read().strip().splitlines()[-1]); print('q=$q L=$L', round(d['value']/1e6,3), 'M q/s', d['p50_ms'], d['p50_ms_serial'])"
done; done
