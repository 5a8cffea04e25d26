#!/bin/bash
# finalize1 phase trace at configs[2] (serial)
set -u
O=gpurun_out/r02u; mkdir -p $O
BB_SELECT_TRACE=1 timeout -k 10 120 python3 tools/scale_bench.py --cases c3 --seconds 0.2 > $O/c3d.jsonl 2> $O/c3d.err || exit 1
grep "finalize trace" $O/c3d.err | tail -3
grep "select trace" $O/c3d.err | tail -3
