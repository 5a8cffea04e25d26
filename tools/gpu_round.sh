#!/bin/bash
# parity tests -> bench -> probes; stop at any abnormal exit
set -u
mkdir -p gpurun_out
bash tools/gpu_check.sh; rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
for t in scan_probe; do
  if [ -x tools/$t ]; then
    timeout -k 10 200 ./tools/$t > gpurun_out/$t.jsonl 2> gpurun_out/$t.err; rc=$?
    echo "$t rc=$rc"; cat gpurun_out/$t.jsonl; tail -3 gpurun_out/$t.err
    [ $rc -ne 0 ] && exit $rc
  fi
done
exit 0
