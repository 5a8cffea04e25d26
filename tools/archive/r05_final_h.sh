# Round-5 final evidence after the rank-0 fold (re-run of r05_final_e1.sh): smoke(), the whole -m gpu suite, configs[3] / configs[4] (bench
# line + inflight-1 rocprof stats + FETCH/WRITE passes) and the shard lines.
set -u
T=r05fh
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -5 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
cp gpurun_out/parity_gates.json gpurun_out/$T/parity_gates.json
bash tools/evidence_run.sh $T c4 c5 || exit $?
timeout -k 10 300 python -u tools/scale_bench.py --cases c4-shard,c4-full,c5-shard --seconds 3 --out gpurun_out/$T/scale.jsonl > gpurun_out/$T/scale.log 2>&1 || exit $?
