"""Rescored rows per query of the list select at configs[1] (VERDICT r03 item 3's counter), on
the GPU box: the list select's BB_SELECT_TRACE probe (csrc/api.hip) prints per batch the mean
candidates, overflowed-list items and rank-0 items rescored per query row.  Run as
    BB_AB=1 BB_SELECT_TRACE=1 python tools/rescore_count.py  2> trace.log
and the stderr lines carry the counts; stdout gets one JSON summary line parsed from them."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, os.path.join(ROOT, "brickbrain-rec-engine_amd"))
    sys.path.insert(0, ROOT)
    import torch
    import brickrec
    from bench import unit_rows_torch
    dev = torch.device("cuda", 0)
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(unit_rows_torch(25216, 384, 1234, dev))
    for seed in range(5):
        idx.search("semantic", 50, q_rows=unit_rows_torch(256, 384, 77 + seed, dev))
    torch.cuda.synchronize()


def main():
    if os.environ.get("RC_CHILD"):
        child()
        return
    env = dict(os.environ, BB_AB="1", BB_SELECT_TRACE="1", RC_CHILD="1")
    p = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True,
                       timeout=300)
    lines = [ln for ln in p.stderr.splitlines() if "list select trace" in ln]
    rows = []
    for ln in lines:
        m = re.search(r"cands ([\d.]+) ovf items ([\d.]+) r0 items ([\d.]+)", ln)
        if m:
            c, o, r = map(float, m.groups())
            rows.append(c + o + r)
    print(json.dumps({"workload": "configs[1]: 25,216 x 384 f32, B=256, k=50 (K_int 51), 5 batches",
                      "rescored_rows_per_query": rows, "mean": sum(rows) / max(len(rows), 1),
                      "trace_lines": lines}))
    return 0 if rows else 1


if __name__ == "__main__":
    sys.exit(main())
