set -u
T=r05r
mkdir -p gpurun_out/$T
timeout -k 10 240 ./tools/scan4_probe 02 > gpurun_out/$T/probe.jsonl 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_scan4.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread -k "not c4_10M" > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -2 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/scale_bench.py --cases c4-shard,c4-full --seconds 3 --out gpurun_out/$T/scale.jsonl > gpurun_out/$T/scale.log 2>&1 || exit $?
bash tools/gpu_run.sh ${T}4 bench --workload c4 --steps 20 --warmup 3 --no-sweep || exit $?
