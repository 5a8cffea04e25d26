"""Streaming top-K diagnostics on one GPU: does the streaming pass finish without a candidate
region overflow (and so without the slab-path rerun) at the BASELINE.json scales?

    BB_STREAM_DEBUG=1 python tools/stream_diag.py [--cases 1000000:384:bf16:1024:100,...]
Prints per case: launches per search by kernel family and the wall time of one search; the
library prints the region statistics to stderr when a region overflows.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brickbrain-rec-engine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="125000:768:bf16:1024:100,1000000:768:bf16:1024:100,"
                                       "1250000:384:bf16:1024:100,300000:384:bf16:1024:100")
    args = ap.parse_args()
    import torch
    import brickrec
    from scale_bench import unit_rows
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for c in args.cases.split(","):
        n, d, dt, B, k = c.split(":")
        n, d, B, k = int(n), int(d), int(B), int(k)
        x = unit_rows(n, d, 1234, dev)
        idx = brickrec.ItemIndex(device=0, dtype=dt)
        idx.upload_items(x, prenormalized=True)
        del x
        q = unit_rows(B, d, 4321, dev)
        idx.set_option("stream", 1)
        idx.search("semantic", k, q_rows=q)
        torch.cuda.synchronize()
        idx.set_profiling(True)
        t0 = time.perf_counter()
        idx.search("semantic", k, q_rows=q)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        prof = idx.profile()
        idx.set_profiling(False)
        print(json.dumps({"case": c, "ms": round(1e3 * el, 3),
                          "launches": {kk: v["launches"] for kk, v in prof.items() if v["launches"]},
                          "us": {kk: round(1e3 * v["ms"], 1) for kk, v in prof.items() if v["launches"]}}),
              flush=True)
        idx.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
