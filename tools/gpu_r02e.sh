set -o pipefail
mkdir -p gpurun_out/r02e
for abl in 4 5 6 7; do
  BB_RR_ABL=$abl timeout -k 10 120 python -u tools/scale_bench.py --cases c2-B1,c2-B256 --seconds 0.5 > gpurun_out/r02e/abl$abl.jsonl 2> gpurun_out/r02e/abl$abl.err || exit $?
done
BB_NO_RR=1 timeout -k 10 120 python -u tools/scale_bench.py --cases c2-B1,c2-B256 --seconds 0.5 > gpurun_out/r02e/norr.jsonl 2> gpurun_out/r02e/norr.err
