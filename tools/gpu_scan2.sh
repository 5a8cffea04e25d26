#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/scan_probe > gpurun_out/scan_probe2.jsonl 2>&1; rc=$?
echo "probe rc=$rc"; cat gpurun_out/scan_probe2.jsonl
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_check.sh
