#!/bin/bash
set -u
mkdir -p gpurun_out/sabl
for a in 0 1 2 4 8; do
  BB_SELECT_ABLATE=$a timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu ${BENCH_ARGS:-} > gpurun_out/sabl/a$a.log 2>&1; rc=$?
  echo "abl=$a rc=$rc $(grep -o '"kernels_us_per_step": {[^}]*}' gpurun_out/sabl/a$a.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
