#!/bin/bash
# GPU-box check: parity tests, then a short bench.  Stops at any abnormal exit.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"; tail -20 gpurun_out/bench.log
exit $rc2
