set -o pipefail
mkdir -p gpurun_out/r02h
timeout -k 10 300 python -u -m pytest tests/test_gpu_rerank.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02h/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/scale_bench.py --cases c2-B1,c2-B256,c2-B1024,c2-B4096,c3 --seconds 0.5 --inflight 3 > gpurun_out/r02h/sweep.jsonl 2> gpurun_out/r02h/sweep.err
