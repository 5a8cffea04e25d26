#!/bin/bash
# select-phase traces (BB_SELECT_TRACE) of the re-rank selects at configs[1], B=1024/4096 and configs[2]
set -u
O=gpurun_out/r02r; mkdir -p $O
for c in c2-B256 c2-B1024 c2-B4096 c3; do
  BB_SELECT_TRACE=1 timeout -k 10 120 python3 tools/scale_bench.py --cases $c --seconds 0.2 > $O/$c.jsonl 2> $O/$c.err; rc=$?
  echo "$c rc=$rc"; grep "trace" $O/$c.err | tail -4; [ $rc -ne 0 ] && { tail -5 $O/$c.err; exit $rc; }
done
exit 0
