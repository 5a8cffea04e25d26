set -u
T=r05w
mkdir -p gpurun_out/$T
timeout -k 10 120 ./tools/scan4_list_probe cf > gpurun_out/$T/cf.jsonl 2>&1 || exit $?
timeout -k 10 120 ./tools/scan4_list_probe > gpurun_out/$T/content.jsonl 2>&1 || exit $?
