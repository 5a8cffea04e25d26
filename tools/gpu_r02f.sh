set -o pipefail
mkdir -p gpurun_out/r02f
for abl in 4; do
  BB_RR_ABL=$abl timeout -k 10 120 python -u tools/scale_bench.py --cases c2-B1,c2-B256 --seconds 0.3 > gpurun_out/r02f/abl$abl.jsonl 2> gpurun_out/r02f/abl$abl.err || exit $?
done
