# Round-5 evidence, part A: the whole -m gpu suite (gate counts -> gpurun_out/parity_gates.json),
# then configs[3] / configs[4] (bench line + inflight-1 rocprof stats + FETCH/WRITE passes) and the
# one-GPU shard lines (tools/scale_bench.py).
set -u
T=r05fa
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
cp gpurun_out/parity_gates.json gpurun_out/$T/parity_gates.json
timeout -k 10 300 python -u tools/scale_bench.py --cases c4-shard,c5-shard --seconds 3 --out gpurun_out/$T/scale.jsonl > gpurun_out/$T/scale.log 2>&1 || exit $?
bash tools/evidence_run.sh $T c4 c5 || exit $?
