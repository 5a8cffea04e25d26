#!/bin/bash
# Phase timeline of the small-batch path on the GPU box (BB_SQ_TRACE): 30 searches per batch
# size, the last trace line of each kept.   bash tools/sq_trace.sh TAG
set -u
O=gpurun_out/$1; mkdir -p $O
for B in 1 4 16; do
  timeout -k 10 120 env BB_AB=1 BB_SQ_TRACE=1 python3 - $B > $O/trace_B$B.log 2>&1 <<'PY' || exit 1
import sys, os
sys.path.insert(0, "brickbrain-rec-engine_amd"); sys.path.insert(0, ".")
import torch, brickrec
from bench import unit_rows_torch
B = int(sys.argv[1]); dev = torch.device("cuda", 0)
idx = brickrec.ItemIndex(dtype="f32"); idx.upload_items(unit_rows_torch(25216, 384, 1234, dev))
q = unit_rows_torch(B, 384, 9, dev)
for _ in range(30):
    idx.search("semantic", 10 if B == 1 else 50, q_rows=q)
torch.cuda.synchronize()
PY
  grep "sq trace" $O/trace_B$B.log | tail -1
done
