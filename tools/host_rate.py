"""Host enqueue rate vs device rate of the configs[1] step (3 lanes in flight): is the
in-flight throughput bound by the host's launch overhead?"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brickbrain-rec-engine_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import brickrec
    from bench import unit_rows_torch
    dev = torch.device("cuda", 0)
    x = unit_rows_torch(25216, 384, 1234, dev)
    for B in (256, 1024):
        lanes = []
        for j in range(3):
            idx = brickrec.ItemIndex(dtype="f32")
            idx.upload_items(x)
            s = torch.cuda.Stream(dev)
            run, _ = idx.prepared_search("semantic", 50, q_rows=unit_rows_torch(B, 384, 9 + j, dev), stream=s)
            lanes.append((idx, s, run))
        for i in range(60):
            lanes[i % 3][2]()
        torch.cuda.synchronize()
        n = 600
        t0 = time.perf_counter()
        for i in range(n):
            lanes[i % 3][2]()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        # device-only rate: the same steps with the host far ahead (queue pre-filled)
        print(json.dumps({"B": B, "host_us_per_step": round(1e6 * (t1 - t0) / n, 2),
                          "wall_us_per_step": round(1e6 * (t2 - t0) / n, 2),
                          "qps": round(B * n / (t2 - t0), 1)}), flush=True)
        for ln in lanes:
            ln[0].close()


if __name__ == "__main__":
    main()
