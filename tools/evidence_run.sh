# Evidence pass on the GPU box: per workload the bench.py line (with cpu_baseline), then
# rocprofv3 --kernel-trace --stats of `bench.py --inflight 1` — one batch at a time, so the
# kernel averages are not inflated by other lanes' batches and match the bench line's
# HIP-event kernel times (roofline.kernel_us) — then the FETCH_SIZE / WRITE_SIZE passes.
#   bash tools/evidence_run.sh TAG [workloads...]      (default: c2 c3 c4 c5)
set -e
T=${1:-r04}; shift || true
WL=${@:-c2 c3 c4 c5}
O=gpurun_out/$T; mkdir -p $O
R=$(pwd)
for w in $WL; do
  timeout -k 10 420 python3 bench.py --workload $w > $O/bench_$w.log 2>&1
  tail -1 $O/bench_$w.log | cut -c1-300
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$w" -o run \
      --output-format csv -- python3 "$R/bench.py" --no-cpu --no-sweep --inflight 1 --workload $w > "$R/$O/prof_$w.log" 2>&1 )
  echo "prof $w ok"
  if [ "$w" = c2 ] || [ "$w" = c3 ]; then
    # cold-MALL twin: the 256 MiB Infinity Cache flushed (640 MiB fill)
    # before every timed step; the fill kernel appears in the stats beside the search's
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_cold_$w" -o run \
        --output-format csv -- python3 "$R/bench.py" --no-cpu --no-sweep --inflight 1 --mall-flush --steps 200 --warmup 20 \
        --workload $w > "$R/$O/prof_cold_$w.log" 2>&1 )
    echo "prof cold $w ok"
  fi
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d "$R/$O/pmc_$w/p$i" -o run \
        --output-format csv -- python3 "$R/bench.py" --steps 30 --warmup 5 --no-cpu --no-sweep --inflight 1 --workload $w \
        > "$R/$O/pmc_${w}_p$i.log" 2>&1 )
  done
  python3 "$R/tools/pmc_summary.py" "$R/$O/pmc_$w" > "$R/$O/pmc_${w}_summary.json"
  echo "pmc $w ok"
done
