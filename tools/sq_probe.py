"""Small-batch latency probe (run under rocprofv3 --kernel-trace to split kernel time from
launch gaps): per case, 200 serial searches on one stream, HIP-event p50 printed as JSON.
    python tools/sq_probe.py [variant ...]     (BB_OPT_SMALL_BATCH values; default 1 0)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brickbrain-rec-engine_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import brickrec
    from bench import unit_rows_torch
    dev = torch.device("cuda", 0)
    x = unit_rows_torch(25216, 384, 1234, dev)
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    s = torch.cuda.Stream(dev)
    out = {}
    for v in [int(a) for a in sys.argv[1:]] or [1, 0]:
        idx.set_option("small_batch", v)
        for B, k in ((1, 10), (4, 50), (16, 50)):
            q = unit_rows_torch(B, 384, 7 + B, dev)
            run, _ = idx.prepared_search("semantic", k, q_rows=q, stream=s)
            for _ in range(20):
                run()
            torch.cuda.synchronize()
            ev = []
            for _ in range(200):
                a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                run()
                e.record(s)
                ev.append((a, e))
                torch.cuda.synchronize()   # one at a time: idle before each
            out[f"v{v}_B{B}"] = round(float(np.median([a.elapsed_time(e) for a, e in ev])) * 1e3, 2)
            if os.environ.get("SQ_PROBE_GRAPH"):  # the same search captured once, replayed
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    run()
                torch.cuda.synchronize()
                ev = []
                for _ in range(200):
                    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    g.replay()
                    e.record(s)
                    ev.append((a, e))
                    torch.cuda.synchronize()
                out[f"v{v}_B{B}_graph"] = round(float(np.median([a.elapsed_time(e) for a, e in ev])) * 1e3, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
