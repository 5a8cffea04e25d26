set -u
T=${1:-r05c}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -4 gpurun_out/$T/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --workload c3 --no-cpu --steps 200 --warmup 20 > gpurun_out/$T/bench_c3.json 2> gpurun_out/$T/bench_c3.err || exit $?
timeout -k 10 300 python3 bench.py --no-cpu --steps 200 --warmup 20 > gpurun_out/$T/bench_c2.json 2> gpurun_out/$T/bench_c2.err || exit $?
T=$T python3 - <<'PY'
import json,sys
for w in ('c3','c2'):
    d=json.loads(open(f'gpurun_out/'+sys.argv[1] if False else f'gpurun_out/{__import__("os").environ.get("T","r05c")}/bench_{w}.json').read().strip().splitlines()[-1])
    print(w, round(d['value']/1e6,3), 'M q/s serial', d['p50_ms_serial'], d['kernels_us_per_step'], 'frac', d['roofline']['frac'])
    if 'gpu_batch_sweep' in d: print([(s['B'], s['p50_ms_serial']) for s in d['gpu_batch_sweep']]); print(d.get('request_latency'))
PY
