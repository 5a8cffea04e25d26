# Shard-size A/B on one GPU: the two-level streaming bound forced on vs
# auto, and other pilot sizes, for the configs[3] / [4] 8-GPU shards.  Output: gpurun_out/$1/.
set -u
T=${1:-r06au}
O=gpurun_out/$T; mkdir -p $O
for r in -1 1; do
  timeout -k 10 300 python3 tools/scale_bench.py --cases c4-shard,c5-shard --refine $r --out $O/scale.jsonl > $O/s$r.log 2>&1 || exit 1
done
for p in 4 6; do
  BB_AB=1 BB_PILOT_DIV=$p timeout -k 10 300 python3 tools/scale_bench.py --cases c4-shard --out $O/scale_pilot$p.jsonl > $O/p$p.log 2>&1 || exit 1
done
python3 - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/scale*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        print(f.split("/")[-1], d["case"], d.get("refine_opt"), d["ms_per_batch"], d["kernels_us_per_batch"])
PY
