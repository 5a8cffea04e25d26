# Round-5 evidence, part B: smoke(), configs[1] / configs[2] (bench line + inflight-1 rocprof stats
# + FETCH/WRITE passes), the driver's own configs[1] command three times, SQ counters of
# configs[2] after this round's changes, and the plan / request latencies.
set -u
T=r05fb
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -5 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
bash tools/evidence_run.sh $T c2 c3 || exit $?
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T/driver_cmd_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/$T/driver_cmd_$r.log | cut -c1-200
done
timeout -k 10 300 python -u tools/plan_latency.py > gpurun_out/$T/plan_latency.jsonl 2> gpurun_out/$T/plan_latency.err || exit $?
bash tools/gpu_run.sh ${T}_sq pmc --workload c3 || exit $?
