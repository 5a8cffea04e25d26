set -u
T=r05q
mkdir -p gpurun_out/$T
timeout -k 10 300 ./tools/scan4_probe > gpurun_out/$T/probe.jsonl 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_rerank.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_stream.py -m gpu -x -q --timeout 180 --timeout-method thread -k "not c4_10M" > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -2 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_run.sh ${T}3 bench --workload c3 --steps 20 --warmup 3 --no-sweep || exit $?
bash tools/gpu_run.sh ${T}5 bench --workload c5 --steps 20 --warmup 3 --no-sweep || exit $?
bash tools/gpu_run.sh ${T}2 bench --steps 300 --warmup 30 --no-sweep || exit $?
