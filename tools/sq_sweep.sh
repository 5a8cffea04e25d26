#!/bin/bash
# Small-batch A/B on the GPU box: parity tests of the small-batch path, then bench.py's batch
# sweep once per BB_SQ variant (0 = large-batch path, 1 = small-batch + merge launch,
# 2 = small-batch, merge in the last workgroup).  Output: gpurun_out/TAG/.
set -u
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_small_batch.py tests/test_gpu_rerank.py -x -q --timeout 120 \
  --timeout-method thread > $O/sq.log 2>&1; rc=$?; tail -3 $O/sq.log; [ $rc -ne 0 ] && exit $rc
for v in "$@"; do
  timeout -k 10 300 env BB_AB=1 BB_SQ=$v python3 bench.py --no-cpu --steps 200 --warmup 20 > $O/bench_sq$v.log 2>&1 || exit 1
  python3 - $O/bench_sq$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], round(d["value"] / 1e6, 3), d["p50_ms_serial"], d["kernels_us_per_step"],
      [(s["B"], s["p50_ms_serial"], round(s["queries_per_s_inflight3"] / 1e6, 3)) for s in d["gpu_batch_sweep"]],
      d.get("request_latency", {}).get("p50_ms_serial"))
PY
done
