set -o pipefail
mkdir -p gpurun_out/r02i
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/r02i/gpu_all.log 2>&1; rc=$?
echo "tests rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/r02i/bench.log 2>&1; echo "bench rc=$?"
