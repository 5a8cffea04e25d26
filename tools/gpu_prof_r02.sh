#!/bin/bash
# Round-2 evidence: per workload (c2 = configs[1], c3 = configs[2], c4 / c5 = configs[3] / [4]
# on one GPU) a rocprofv3 kernel-trace --stats run and FETCH_SIZE / WRITE_SIZE PMC passes of
# the same bench command, then the default bench line (CPU baselines included).
# usage: bash tools/gpu_prof_r02.sh TAG [workloads...]
set -u
TAG=$1; shift
WL=${@:-c2 c3 c4 c5}
R=$(pwd)
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for w in $WL; do
  case $w in c4|c5) st=4;; *) st=40;; esac
  args="--workload $w --steps $st --warmup 3 --no-cpu --no-sweep --inflight 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$w" -o run --output-format csv -- python3 "$R/bench.py" $args > "$O/prof_$w.log" 2>&1
  rc=$?; echo "stats $w rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/prof_$w.log"; exit $rc; }
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d "$O/pmc_$w/p$i" -o run --output-format csv -- python3 "$R/bench.py" $args > "$O/pmc_${w}_p$i.log" 2>&1
    rc=$?; echo "pmc $w $grp rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/pmc_${w}_p$i.log"; exit $rc; }
  done
  python3 "$R/tools/pmc_summary.py" "$O/pmc_$w" > "$O/pmc_$w/summary.json"
done
cd "$R"
timeout -k 10 400 python3 bench.py > "$O/bench.log" 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 "$O/bench.log"
exit $rc
