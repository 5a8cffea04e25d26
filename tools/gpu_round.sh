#!/bin/bash
# parity tests -> tile micro-bench -> bench; stop at any abnormal exit
set -u
mkdir -p gpurun_out
bash tools/gpu_check.sh; rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -x tools/gemm_tiles ]; then
  timeout -k 10 300 ./tools/gemm_tiles 20 > gpurun_out/gemm_tiles.jsonl 2> gpurun_out/gemm_tiles.err; rc=$?
  echo "gemm_tiles rc=$rc"; cat gpurun_out/gemm_tiles.jsonl; tail -3 gpurun_out/gemm_tiles.err
fi
exit $rc
