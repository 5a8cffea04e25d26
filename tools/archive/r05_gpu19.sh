set -u
T=r05ab2
mkdir -p gpurun_out/$T
for r in 1 2; do
  for lib in tree tools/ab/lib_b0ef42e.so tools/ab/lib_ab2556d.so; do
    L=X=1; [ "$lib" != tree ] && L=BRICKREC_LIB=$(pwd)/$lib
    nm=$(basename $lib)
    timeout -k 10 200 env $L python -u tools/scale_bench.py --cases c5-full --seconds 3 --out gpurun_out/$T/${nm}_$r.jsonl > gpurun_out/$T/${nm}_$r.log 2>&1 || exit $?
    python3 -c "
import json
for l in open('gpurun_out/$T/${nm}_$r.jsonl'):
    d=json.loads(l); print('$nm', d['case'], d['ms_per_batch'], d['kernels_us_per_batch'])"
  done
done
