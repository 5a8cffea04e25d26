#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter group per rocprofv3 run, kernel-trace only) over
# configs[1] and configs[2] on the final round-2 build -> profiles/pmc_traffic.json
set -u
R=$(pwd); O="$R/gpurun_out/r02zi"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for w in c2 c3; do
  i=0; mkdir -p "$O/pmc_$w"
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp -d "$O/pmc_$w/p$i" -o run --output-format csv -- python3 "$R/bench.py" --workload $w --steps 30 --warmup 5 --no-cpu --no-sweep --inflight 1 > "$O/pmc_$w/p$i.log" 2>&1
    rc=$?; echo "$w pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/pmc_$w/p$i.log"; exit $rc; }
  done
  python3 "$R/tools/pmc_summary.py" "$O/pmc_$w" > "$O/pmc_$w/summary.json" || exit 1
done
