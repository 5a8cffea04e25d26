# one PMC pass (VALU / SALU / MFMA instruction counts, waves) + a bench line of WORKLOAD
set -u
T=$1; W=$2; shift 2
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
timeout -k 10 300 env BB_AB=1 "$@" python3 bench.py --workload $W --no-cpu --no-sweep --steps 300 --warmup 30 > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('$W', round(d['value']/1e6,4), 'M q/s', d.get('p50_ms_serial'), d['kernels_us_per_step'], 'frac', d['roofline']['frac'])"
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 env BB_AB=1 "$@" rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES -d $O/pmc -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 30 --warmup 5 --no-cpu --no-sweep --inflight 1 > $O/pmc.log 2>&1 ) || exit $?
python3 $R/tools/pmc_summary.py $O/pmc > $O/pmc_summary.json
python3 -c "
import json
d=json.load(open('$O/pmc_summary.json'))
for k,v in d.items():
    if v.get('_dispatches',0) >= 20 and 'bb::' in k: print(k[:50], {c: round(x/max(v.get('SQ_WAVES',1),1),1) for c,x in v.items() if c.startswith('SQ_INSTS')}, 'waves', v.get('SQ_WAVES'))"
