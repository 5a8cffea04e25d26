set -u
mkdir -p gpurun_out/r05b
timeout -k 10 120 ./tools/launch_cost > gpurun_out/r05b/launch_cost.jsonl 2>&1; rc=$?
cat gpurun_out/r05b/launch_cost.jsonl
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_run.sh r05b_c3 pmc --workload c3 || exit $?
bash tools/gpu_run.sh r05b_c2 pmc --workload c2 || exit $?
