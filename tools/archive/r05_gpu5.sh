set -u
mkdir -p gpurun_out/r05e
timeout -k 10 120 ./tools/percu_probe > gpurun_out/r05e/percu.jsonl 2>&1 || exit $?
cat gpurun_out/r05e/percu.jsonl
bash tools/r05_gpu4.sh r05d
