# pilot-size A/B on the final build (BB_PILOT_DIV, one box): the configs[3] shard and full index
set -u
O=gpurun_out/r05pilot; mkdir -p $O
for rep in 1 2; do
  for d in 6 8 12; do
    BB_AB=1 BB_PILOT_DIV=$d timeout -k 10 200 python3 tools/scale_bench.py --cases c4-shard --seconds 2 --out $O/shard_div${d}_$rep.jsonl > $O/shard_div${d}_$rep.log 2>&1 || exit $?
  done
  for d in 12 16 24; do
    BB_AB=1 BB_PILOT_DIV=$d timeout -k 10 200 python3 tools/scale_bench.py --cases c4-full --seconds 3 --out $O/full_div${d}_$rep.jsonl > $O/full_div${d}_$rep.log 2>&1 || exit $?
  done
done
