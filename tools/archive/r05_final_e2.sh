# Round-5 final evidence (2/2): configs[1] / configs[2] (bench line + inflight-1 rocprof stats +
# FETCH/WRITE passes), the driver's own configs[1] command twice, plan / request latencies.
set -u
T=r05fe
mkdir -p gpurun_out/$T
bash tools/evidence_run.sh $T c2 c3 || exit $?
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T/driver_cmd_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/$T/driver_cmd_$r.log | cut -c1-200
done
timeout -k 10 300 python -u tools/plan_latency.py > gpurun_out/$T/plan_latency.jsonl 2> gpurun_out/$T/plan_latency.err || exit $?
