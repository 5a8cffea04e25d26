#!/bin/bash
# in-flight lanes on the views' own streams (bb_get_stream) vs torch pool streams, 3/4/5 lanes
set -u
O=gpurun_out/r02v4; mkdir -p $O
for rep in 1 2; do
  for cfg in "X=1:--inflight 3" "X=1:--inflight 4" "X=1:--inflight 5" "BB_BENCH_TORCH_STREAMS=1:--inflight 3"; do
    e=${cfg%%:*}; args=${cfg#*:}; tag=$(echo $e$args | tr -d ' -=')
    timeout -k 10 200 env $e python3 bench.py --no-cpu --no-sweep $args > $O/b_${tag}_$rep.log 2>&1 || { tail -5 $O/b_${tag}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${tag}_$rep.log').read().strip().splitlines()[-1]); print('$e $args'.ljust(40), round(d['value']/1e6,3), d['p50_ms'], d['p50_ms_serial'])"
  done
done
for cfg in "X=1:--inflight 3" "X=1:--inflight 4" "BB_BENCH_TORCH_STREAMS=1:--inflight 3"; do
  e=${cfg%%:*}; args=${cfg#*:}; tag=$(echo $e$args | tr -d ' -=')
  timeout -k 10 200 env $e python3 bench.py --workload c3 --steps 300 --no-cpu $args > $O/c3_${tag}.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/c3_${tag}.log').read().strip().splitlines()[-1]); print('c3 $e $args'.ljust(40), round(d['value']/1e6,3), d['p50_ms_serial'])"
done
