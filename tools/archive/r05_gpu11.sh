set -u
T=r05t
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -2 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for m in 0 1 2; do
    BB_AB=1 BB_SPIN_WAIT=$m timeout -k 10 200 python -u tools/scale_bench.py --cases c4-shard,c2-B1 --seconds 2 --out gpurun_out/$T/spin$m.r$r.jsonl > gpurun_out/$T/spin$m.r$r.log 2>&1 || exit $?
  done
done
