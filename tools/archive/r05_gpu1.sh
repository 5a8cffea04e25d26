set -u
mkdir -p gpurun_out/r05a
timeout -k 10 600 python -u -m pytest tests/test_gpu_small_batch.py::test_plan_refused_on_streaming_falls_back tests/test_gpu_small_batch.py::test_destroyed_handle_is_an_error tests/test_gpu_stream.py -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/r05a/tests.log 2>&1; rc=$?
tail -5 gpurun_out/r05a/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/plan_latency.py > gpurun_out/r05a/plan_latency.jsonl 2>&1; rc=$?
cat gpurun_out/r05a/plan_latency.jsonl
exit $rc
