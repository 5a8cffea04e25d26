set -u
T=r05v
mkdir -p gpurun_out/$T
for r in 1 2 3 4; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T/driver_cmd_$r.log 2>&1 || exit $?
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/driver_cmd_$r.log') if l.startswith('{')][-1])
print(round(d['value']/1e6,3), d['ms_per_step'], d['p50_ms'], d['p50_ms_serial'])"
done
