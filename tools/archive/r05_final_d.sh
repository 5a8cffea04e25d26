# Round-5 evidence, part D: configs[4] on the final build (bench line + inflight-1 rocprof
# stats + FETCH/WRITE passes).
set -u
T=r05fd
mkdir -p gpurun_out/$T
bash tools/evidence_run.sh $T c5 || exit $?
