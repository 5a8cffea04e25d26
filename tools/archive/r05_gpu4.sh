set -u
T=${1:-r05d}
bash tools/gpu_run.sh ${T} prof --workload c3 --inflight 1 --steps 100 --warmup 10 || exit $?
bash tools/gpu_run.sh ${T} pmc --workload c3 || exit $?
