#!/bin/bash
# final-build bench lines + rocprofv3 stats of the sharded large-index workloads (configs[3] / [4], one GPU)
set -u
O=gpurun_out/r02zk; mkdir -p $O
R=$(pwd); cd /tmp && export TMPDIR=/tmp
for w in c4 c5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$w" -o run --output-format csv -- python3 "$R/bench.py" --workload $w --steps 10 --warmup 2 --no-cpu > "$R/$O/bench_$w.log" 2>&1; rc=$?
  echo "$w rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/$O/bench_$w.log"; exit $rc; }
  python3 -c "import json; d=json.loads([l for l in open('$R/$O/bench_$w.log') if l.startswith('{')][-1]); print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('bound'))"
done
