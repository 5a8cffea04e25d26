set -u
T=r05u
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_scan4.py tests/test_gpu_configs.py tests/test_gpu_small_batch.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -2 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tools/scale_bench.py --cases c4-shard,c5-shard --seconds 3 --out gpurun_out/$T/scale.r$r.jsonl > gpurun_out/$T/scale.r$r.log 2>&1 || exit $?
done
