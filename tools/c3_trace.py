"""Phase timelines of configs[2] (hybrid B=1024 + mask + rated, the bench's own inputs) on the GPU
box: the list select's and finalize1's BB_SELECT_TRACE lines (in-kernel s_memrealtime stamps).
    python tools/c3_trace.py 2> trace.log     (sets BB_AB=1 BB_SELECT_TRACE=1 itself)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    import faulthandler
    faulthandler.enable()
    sys.path.insert(0, os.path.join(ROOT, "brickbrain-rec-engine_amd"))
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import brickrec
    import bench
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(2024)
    extra = {"f": rng.normal(0.0, 0.1, (bench.N_ITEMS, 50)).astype(np.float32),
             "parts": rng.integers(1, 6000, bench.N_ITEMS).astype(np.int32),
             "year": rng.integers(1949, 2025, bench.N_ITEMS).astype(np.int16),
             "theme": rng.integers(0, 400, bench.N_ITEMS).astype(np.int32)}
    x = bench.unit_rows_torch(bench.N_ITEMS, bench.DIM, 1234, dev)
    print("uploading", flush=True)
    base = bench.make_base(brickrec, "c3", x, 0, "f32", extra)
    print("lane", flush=True)
    _, _, run, _, _ = bench.make_lane(brickrec, "c3", base, 1024, 0, dev, 0, 0, 1, extra)
    print("searching", flush=True)
    for _ in range(4):
        run.prof_run()   # bb_search itself (a plan records its launches once; the traces sync per search)
    torch.cuda.synchronize()


def main():
    os.environ["BB_AB"] = "1"  # (read by the library at its first search)
    if "--scan" in sys.argv:
        os.environ["BB_SCAN_TRACE"] = "1"      # the list scans' phase stamps (scan4)
    elif "--no-trace" not in sys.argv:
        os.environ["BB_SELECT_TRACE"] = "1"
    child()
    print("c3 trace run ok", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
