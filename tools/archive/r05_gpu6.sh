set -u
T=${1:-r05f}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
cp gpurun_out/parity_gates.json gpurun_out/$T/parity_gates.json 2>/dev/null
for w in c3 c2; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu --no-sweep --steps 300 --warmup 30 > gpurun_out/$T/bench_$w.json 2> gpurun_out/$T/bench_$w.err || exit $?
done
timeout -k 10 400 python3 bench.py --workload c5 --no-cpu --steps 5 --warmup 2 > gpurun_out/$T/bench_c5.json 2> gpurun_out/$T/bench_c5.err || exit $?
for w in c3 c2 c5; do
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/$T/bench_$w.json').read().strip().splitlines()[-1])
print('$w', round(d['value']/1e6,4), 'M q/s', d.get('p50_ms_serial'), d['kernels_us_per_step'], 'frac', d['roofline']['frac'])"
done
