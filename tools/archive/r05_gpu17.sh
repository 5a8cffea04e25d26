set -u
T=r05pf2
mkdir -p gpurun_out/$T
for pf in 2 3 4; do
  timeout -k 10 200 ./tools/scan4_probe_pf$pf 02 > gpurun_out/$T/probe_pf$pf.jsonl 2>&1 || exit $?
done
