# round-2 GPU check: the full-shape config parity tests, then the whole -m gpu suite
set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r02a/configs.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r02a/gpu_all.log 2>&1
