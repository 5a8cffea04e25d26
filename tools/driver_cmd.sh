# The driver's own bench command (bench.py --gpus 1 --steps 20 --warmup 5), N times in a row:
# the line the round-end BENCH record reads, with its spread.  Output: gpurun_out/$1/.
set -u
T=${1:-r06drv}; N=${2:-3}
O=gpurun_out/$T; mkdir -p $O
for i in $(seq 1 $N); do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b$i.log 2>&1 || exit 1
  grep "^{" $O/b$i.log | tail -1 >> $O/driver_cmd.jsonl
done
python3 - "$O/driver_cmd.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["value"], d["ms_per_step"], d["p50_ms_serial"], d["roofline"]["frac"])
PY
