# Final-evidence pass: bench.py line (with cpu_baseline) and rocprofv3 --kernel-trace --stats per workload.
set -e
O=gpurun_out/${1:-r03h}; mkdir -p $O
R=$(pwd)
for w in c2 c3 c4 c5; do
  st=""
  timeout -k 10 420 python3 bench.py --workload $w $st > $O/bench_$w.log 2>&1
  tail -1 $O/bench_$w.log | cut -c1-300
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$w" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --no-sweep --workload $w $st > "$R/$O/prof_$w.log" 2>&1 )
  echo "prof $w ok"
done
