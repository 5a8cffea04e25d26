# configs[3] 125K x 768 shard: pilot-size sweep (BB_PILOT_DIV, A/B knob) on one box
#   bash tools/pilot_sweep.sh OUTDIR [divs...]
set -e
O=${1:-gpurun_out/pilot}; shift || true
DIVS=${@:-8 12 16}
mkdir -p $O
for d in $DIVS; do
  BB_AB=1 BB_PILOT_DIV=$d timeout -k 10 200 python3 tools/scale_bench.py --cases c4-shard --seconds 2 > $O/div$d.log 2>&1
  echo "div $d: $(grep c4-shard $O/div$d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_batch"], d["kernels_us_per_batch"])')"
done
