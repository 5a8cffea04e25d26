"""Serial request latency through a bb_plan vs bb_search: per case the
p50 of HIP events around one call on an idle stream (what bench.py's request_latency and
gpu_batch_sweep report) and the host time of the call itself (perf_counter around it)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brickbrain-rec-engine_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import brickrec
    from bench import unit_rows_torch, N_ITEMS, DIM
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(77)
    x = unit_rows_torch(N_ITEMS, DIM, 1234, dev)
    f = rng.normal(0.0, 0.1, (N_ITEMS, 50)).astype(np.float32)
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    idx.upload_cf(f)
    mask = torch.from_numpy(brickrec.bits_from_bool(rng.random(N_ITEMS) < 0.1).view(np.int32)).to(dev)
    rated = np.zeros((1, N_ITEMS), bool)
    rated[0, rng.choice(N_ITEMS, 20, replace=False)] = True
    excl = torch.from_numpy(brickrec.bits_from_bool(rated).view(np.int32)).to(dev)
    liked = torch.tensor([int(rng.integers(N_ITEMS))], device=dev)
    u = torch.from_numpy(rng.normal(0.0, 0.1, (1, 50)).astype(np.float32)).to(dev)
    s = torch.cuda.Stream(dev)
    cases = {"similar_k10": dict(mode="similar", k=10, q_items=liked),
             "retriever_k20": dict(mode="semantic", k=20, q_rows=unit_rows_torch(1, DIM, 991, dev)),
             "cf_k20_rated": dict(mode="cf", k=20, q_cf=u, excl=excl),
             "hybrid_k10_mask_rated": dict(mode="hybrid", k=10, q_items=liked, q_cf=u, mask=mask, excl=excl),
             "semantic_B1_k10": dict(mode="semantic", k=10, q_rows=unit_rows_torch(1, DIM, 555, dev)),
             "semantic_B16_k50": dict(mode="semantic", k=50, q_rows=unit_rows_torch(16, DIM, 556, dev)),
             "semantic_B256_k50": dict(mode="semantic", k=50, q_rows=unit_rows_torch(256, DIM, 557, dev))}
    for name, c in cases.items():
        row = {"case": name}
        for plan in (True, False):
            c2 = dict(c)
            run, _ = idx.prepared_search(c2.pop("mode"), c2.pop("k"), stream=s, plan=plan, **c2)
            for _ in range(20):
                run()
            torch.cuda.synchronize()
            ev, host = [], []
            for _ in range(200):
                a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                t0 = time.perf_counter()
                run()
                host.append(time.perf_counter() - t0)
                e.record(s)
                ev.append((a, e))
                torch.cuda.synchronize()
            tag = "plan" if plan else "search"
            row[f"{tag}_p50_us"] = round(1e3 * float(np.median([a.elapsed_time(e) for a, e in ev])), 2)
            row[f"{tag}_host_us"] = round(1e6 * float(np.median(host)), 2)
            if plan:
                run.close()
        print(json.dumps(row), flush=True)
    idx.close()


if __name__ == "__main__":
    main()
