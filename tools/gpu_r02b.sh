set -o pipefail
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/r02b/gpu_all.log 2>&1 && \
bash tools/gpu_prof_r02.sh r02b c2 c3 c4 c5
