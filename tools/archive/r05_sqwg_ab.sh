# small-batch pass workgroup count A/B (BB_SQ_WG; default 256 = one per CU) on the request latencies
set -u
O=gpurun_out/r05sqwg; mkdir -p $O
for rep in 1 2; do
  for w in 256 512 384 192; do
    BB_AB=1 BB_SQ_WG=$w timeout -k 10 200 python -u tools/plan_latency.py > $O/wg${w}_$rep.jsonl 2> $O/wg${w}_$rep.err || exit $?
  done
done
