set -o pipefail
mkdir -p gpurun_out/r02k
for L in 2 4 6; do
timeout -k 10 200 python -u tools/scale_bench.py --cases c2-B256,c2-B1024 --seconds 0.5 --inflight $L > gpurun_out/r02k/L$L.jsonl 2> gpurun_out/r02k/L$L.err || exit $?
done
