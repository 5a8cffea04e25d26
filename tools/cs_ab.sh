# candidate select A/B on one box: the wave-per-query kernel (default) vs the
# workgroup-per-query kernel (BB_CS_WG=1), over the streaming cases of tools/scale_bench.py
#   bash tools/cs_ab.sh OUTDIR [cases]
set -e
O=${1:-gpurun_out/cs_ab}; C=${2:-c4-shard,c4-full,c5-shard,c5-full}
mkdir -p $O
for v in wave wg; do
  if [ $v = wg ]; then export BB_AB=1 BB_CS_WG=1; else unset BB_CS_WG; export BB_AB=1; fi
  timeout -k 10 400 python3 tools/scale_bench.py --cases $C --seconds 2 > $O/$v.log 2>&1
  python3 - $O/$v.log $v <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        print(sys.argv[2], d["case"], d["ms_per_batch"], d["kernels_us_per_batch"], flush=True)
PY
done
