set -u
T=r05x
mkdir -p gpurun_out/$T
timeout -k 10 120 ./tools/scan4_list_probe cf > gpurun_out/$T/cf.jsonl 2>&1 || exit $?
timeout -k 10 120 ./tools/scan4_list_probe > gpurun_out/$T/content.jsonl 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_rerank.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_scan4.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -2 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_run.sh ${T}3 bench --workload c3 --steps 300 --warmup 30 --no-sweep || exit $?
bash tools/gpu_run.sh ${T}2 bench --steps 300 --warmup 30 --no-sweep || exit $?
timeout -k 10 200 python -u tools/scale_bench.py --cases c5-shard,c4-shard --seconds 3 --out gpurun_out/$T/scale.jsonl > gpurun_out/$T/scale.log 2>&1 || exit $?
