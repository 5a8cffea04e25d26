# Round-5 evidence, part C (after the d = 768 fragment addressing): the whole -m gpu suite,
# configs[3] (bench line + inflight-1 rocprof stats + FETCH/WRITE), the shard lines, the
# configs[1] / configs[2] bench lines and the driver's own configs[1] command twice.
set -u
T=r05fc
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
cp gpurun_out/parity_gates.json gpurun_out/$T/parity_gates.json
bash tools/evidence_run.sh $T c4 || exit $?
timeout -k 10 300 python -u tools/scale_bench.py --cases c4-shard,c4-full,c5-shard --seconds 3 --out gpurun_out/$T/scale.jsonl > gpurun_out/$T/scale.log 2>&1 || exit $?
for w in c2 c3; do
  timeout -k 10 420 python3 bench.py --workload $w > gpurun_out/$T/bench_$w.log 2>&1 || exit $?
  tail -1 gpurun_out/$T/bench_$w.log | cut -c1-200
done
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T/driver_cmd_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/$T/driver_cmd_$r.log | cut -c1-200
done
