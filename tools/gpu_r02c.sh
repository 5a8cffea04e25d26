set -o pipefail
mkdir -p gpurun_out/r02c
timeout -k 10 300 python -u tools/scale_bench.py --cases b2-B1,b2-B256,b2-B1024,b2-B4096,c2-B256 --seconds 1 --inflight 3 > gpurun_out/r02c/b2.jsonl 2> gpurun_out/r02c/b2.err && \
BB_NO_SCAN4=1 timeout -k 10 300 python -u tools/scale_bench.py --cases b2-B256,b2-B1024 --seconds 1 --inflight 3 > gpurun_out/r02c/b2_noscan4.jsonl 2>> gpurun_out/r02c/b2.err
