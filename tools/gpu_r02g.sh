set -o pipefail
mkdir -p gpurun_out/r02g
timeout -k 10 300 python -u -m pytest tests/test_gpu_rerank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02g/rerank.log 2>&1 || exit $?
for abl in 0 1; do
  BB_RR_ABL=$abl timeout -k 10 120 python -u tools/scale_bench.py --cases c2-B1,c2-B256,c2-B1024,c3 --seconds 0.5 --inflight 3 > gpurun_out/r02g/abl$abl.jsonl 2> gpurun_out/r02g/abl$abl.err || exit $?
done
