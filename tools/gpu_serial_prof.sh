#!/bin/bash
# Serial (one batch at a time) rocprofv3 kernel stats of a bench workload: clean per-kernel
# durations without the in-flight lanes' interference.  usage: TAG [bench args...]
set -u
T=$1; shift
R=$(pwd); O="$R/gpurun_out/$T"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/serial" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --no-sweep --inflight 1 --steps 300 --warmup 20 "$@" > "$O/serial.log" 2>&1; rc=$?
echo "serial prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/serial.log"; exit $rc; }
python3 - "$O/serial/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if int(r["Calls"]) >= 100: print(f'{r["Name"][:60]:60s} {r["Calls"]:>6s} {float(r["AverageNs"])/1000:8.2f} us')
PY
