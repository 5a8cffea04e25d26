set -o pipefail
mkdir -p gpurun_out/r02d
timeout -k 10 300 python -u -m pytest tests/test_gpu_rerank.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02d/rerank.log 2>&1; rc=$?
echo "rerank rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/r02d/gpu_all.log 2>&1; rc2=$?
echo "all rc=$rc2"
[ $rc2 -ne 0 ] && [ $rc2 -ne 1 ] && exit $rc2
timeout -k 10 300 python -u tools/scale_bench.py --cases c2-B1,c2-B256,c2-B1024,c2-B4096,c3 --seconds 1 --inflight 3 > gpurun_out/r02d/sweep.jsonl 2> gpurun_out/r02d/sweep.err
echo "sweep rc=$?"
