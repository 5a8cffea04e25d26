set -u
T=r05g
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_rerank.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_small_batch.py -m gpu -x -q --timeout 180 --timeout-method thread -k "not c3_1M and not c4_10M" > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -2 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_run.sh $T bench --workload c3 --steps 300 --warmup 30 --no-sweep -- "X=1" "BB_LS_BITWISE=1" "X=1" "BB_LS_BITWISE=1" || exit $?
bash tools/gpu_run.sh ${T}b bench --steps 300 --warmup 30 --no-sweep -- "X=1" "BB_LS_BITWISE=1" "X=1" "BB_LS_BITWISE=1" || exit $?
