#!/bin/bash
# Alternating A/B of built libraries on one box: bash tools/ab_libs.sh TAG REPS "LIB..." BENCH_ARGS...
# LIB = "tree" (this tree's libbrickrec.so) or a path; prints one summary line per run.
set -u
T=$1; REPS=$2; LIBS=$3; shift 3
R=$(pwd); O="$R/gpurun_out/$T"; mkdir -p "$O"
for rep in $(seq 1 $REPS); do
  for lib in $LIBS; do
    L=X=1; [ "$lib" != tree ] && L=BRICKREC_LIB=$R/$lib
    nm=$(basename "$lib")
    timeout -k 10 300 env $L python3 bench.py --no-cpu --no-sweep "$@" > "$O/${nm}_$rep.log" 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "$lib rc=$rc"; tail -3 "$O/${nm}_$rep.log"; exit $rc; }
    python3 - "$O/${nm}_$rep.log" "$nm" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2].ljust(24), round(d["value"] / 1e6, 3), "M q/s", "serial", d.get("p50_ms_serial"), d.get("kernels_us_per_step"))
PY
  done
done
