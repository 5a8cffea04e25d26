"""Scale sweep on one MI355X: the BASELINE.json shapes beyond bench.py's configs[1] line.

One JSON line per case (queries/s, p50 per batch, per-kernel device time, algorithmic roofline):
  c2-B{1,256,1024,4096}  semantic top-50 over 25,216 x 384 f32               (configs[1] batch sweep)
  c3                     hybrid (liked-set content + CF r=50) + mask, B=1024, top-50, f32 (configs[2])
  c4-shard               125,000 x 768 bf16, B=4096, top-100  (one GPU's shard of configs[3])
  c4-full                1,000,000 x 768 bf16, B=4096, top-100 on one GPU
  c5-shard               1,250,000 x 384 bf16, B=8192, top-100 (one GPU's shard of configs[4] at P=8)
  c5-full                10,000,000 x 384 bf16, B=8192, top-100 on one GPU (P=1 point)

    python tools/scale_bench.py [--cases c2,c3,c4-shard,...] [--seconds 2]
Inputs are synthetic: unit-norm N(0,1) rows, seeds 1234 / 4321; CF factors
N(0, 0.1^2); mask = random bitset at ~10 % density.  Inputs are resident in HBM.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brickbrain-rec-engine_amd"))

BF16_TF, F32_TF, HBM = 2500.0, 157.3, 8000.0

CASES = {
    "c2-B1": dict(n=25216, d=384, B=1, k=50, dtype="f32", mode="semantic"),
    "c2-B256": dict(n=25216, d=384, B=256, k=50, dtype="f32", mode="semantic"),
    "c2-B1024": dict(n=25216, d=384, B=1024, k=50, dtype="f32", mode="semantic"),
    "c2-B4096": dict(n=25216, d=384, B=4096, k=50, dtype="f32", mode="semantic"),
    "c3": dict(n=25216, d=384, B=1024, k=50, dtype="f32", mode="hybrid", r=50),
    "c4-shard": dict(n=125000, d=768, B=4096, k=100, dtype="bf16", mode="semantic"),
    "c4-full": dict(n=1000000, d=768, B=4096, k=100, dtype="bf16", mode="semantic"),
    "c5-shard": dict(n=1250000, d=384, B=8192, k=100, dtype="bf16", mode="semantic"),
    "c5-full": dict(n=10000000, d=384, B=8192, k=100, dtype="bf16", mode="semantic"),
    # an f32 index at scale (MiniLM embeddings are f32): the split-precision streaming scan
    "f32-1M": dict(n=1000000, d=384, B=4096, k=100, dtype="f32", mode="semantic"),
    # bf16 index at the 25K shape (the one-product MFMA scan, no split)
    "b2-B1": dict(n=25216, d=384, B=1, k=50, dtype="bf16", mode="semantic"),
    "b2-B256": dict(n=25216, d=384, B=256, k=50, dtype="bf16", mode="semantic"),
    "b2-B1024": dict(n=25216, d=384, B=1024, k=50, dtype="bf16", mode="semantic"),
    "b2-B4096": dict(n=25216, d=384, B=4096, k=50, dtype="bf16", mode="semantic"),
    # north_star latency points: small batches against the large indexes
    "c4-B1": dict(n=1000000, d=768, B=1, k=100, dtype="bf16", mode="semantic"),
    "c4-B256": dict(n=1000000, d=768, B=256, k=100, dtype="bf16", mode="semantic"),
    "c4-B1024": dict(n=1000000, d=768, B=1024, k=100, dtype="bf16", mode="semantic"),
    "c5-B1": dict(n=10000000, d=384, B=1, k=100, dtype="bf16", mode="semantic"),
    "c5-B256": dict(n=10000000, d=384, B=256, k=100, dtype="bf16", mode="semantic"),
}


def unit_rows(n, d, seed, dev, chunk=1 << 20):
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    out = torch.empty((n, d), dtype=torch.float32, device=dev)
    for i in range(0, n, chunk):
        x = torch.randn((min(chunk, n - i), d), generator=g, device=dev)
        out[i:i + x.shape[0]] = x / x.norm(dim=1, keepdim=True)
    return out


def run_case(name, c, seconds, dev, stream=-1, inflight=1, refine=-1):
    import torch
    import brickrec
    n, d, B, k, dt = c["n"], c["d"], c["B"], c["k"], c["dtype"]
    x = unit_rows(n, d, 1234, dev)
    idx = brickrec.ItemIndex(device=dev.index, dtype=dt)
    idx.upload_items(x, prenormalized=True)
    idx.set_option("stream", stream)
    idx.set_option("stream_refine", refine)
    # extra lanes for the in-flight throughput (bench.py's scheme): own handle, stream, copy
    lanes = []
    for j in range(1, inflight):
        lj = brickrec.ItemIndex(device=dev.index, dtype=dt)
        lj.upload_items(x, prenormalized=True)
        lj.set_option("stream", stream)
        lj.set_option("stream_refine", refine)
        lanes.append(lj)
    del x
    torch.cuda.empty_cache()
    kw = {}
    flops = 2.0 * B * n * d
    es = 4 if dt == "f32" else 2
    nbytes = n * d * es + B * d * 4 + B * k * 8
    if c["mode"] == "hybrid":
        r = c["r"]
        rng = np.random.default_rng(7)
        f = rng.normal(0, 0.1, (n, r)).astype(np.float32)
        idx.upload_cf(f)
        for lj in lanes:
            lj.upload_cf(f)
        mask = rng.random(n) < 0.10
        words = brickrec.engine.bits_from_bool(mask).view(np.int32)
        kw = dict(q_items=torch.from_numpy(rng.integers(0, n, B)).to(dev),
                  q_cf=torch.from_numpy(rng.normal(0, 0.1, (B, r)).astype(np.float32)).to(dev),
                  mask=torch.from_numpy(words).to(dev))
        flops += 2.0 * B * n * r
        nbytes += n * r * 4 + B * r * 4 + (n + 7) // 8
    else:
        kw = dict(q_rows=unit_rows(B, d, 4321, dev))
    s = torch.cuda.current_stream(dev)
    run, _ = idx.prepared_search(c["mode"], k, stream=s, **kw)
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    one = time.perf_counter() - t0
    steps = int(max(3, min(500, seconds / max(one, 1e-6))))
    for _ in range(min(steps // 10 + 1, 20)):
        run()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(s)
        run()
        b.record(s)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    lat = np.array([a.elapsed_time(b) for a, b in ev])
    idx.set_profiling(True)
    ps = min(steps, 50)
    run_p, _ = idx.prepared_search(c["mode"], k, stream=s, plan=False, **kw)   # (a plan's view is not profiled)
    for _ in range(ps):
        run_p()
    torch.cuda.synchronize()
    prof = idx.profile()
    idx.set_profiling(False)
    kern = {kk: round(1e3 * v["ms"] / ps, 2) for kk, v in prof.items() if v["launches"]}
    launches = {kk: v["launches"] // ps for kk, v in prof.items() if v["launches"]}
    gemm_us = kern.get("gemm", 0.0)
    peak = F32_TF if dt == "f32" else BF16_TF
    out = {"case": name, **{kk: v for kk, v in c.items()}, "stream_opt": stream, "refine_opt": refine, "steps": steps,
           "qps": round(B * steps / el, 1), "ms_per_batch": round(1e3 * el / steps, 4),
           "p50_ms": round(float(np.median(lat)), 4),
           "kernels_us_per_batch": kern, "launches_per_batch": launches,
           "alg_tflops_end_to_end": round(flops / (el / steps) / 1e12, 2),
           "alg_tflops_scan": round(flops / (gemm_us * 1e-6) / 1e12, 2) if gemm_us else None,
           "mfma_peak_tflops": peak,
           "frac_end_to_end": round(flops / (el / steps) / 1e12 / peak, 4),
           "alg_bytes": nbytes,
           "hbm_frac_end_to_end": round(nbytes / (el / steps) / 1e9 / HBM, 4)}
    if lanes:
        # `inflight` batches in flight on as many streams, steps alternating between them
        runs = [(s, run)]
        for lj in lanes:
            sj = torch.cuda.Stream(dev)
            runs.append((sj, lj.prepared_search(c["mode"], k, stream=sj, **kw)[0]))
        for i in range(2 * len(runs)):
            runs[i % len(runs)][1]()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            runs[i % len(runs)][1]()
        torch.cuda.synchronize()
        el2 = time.perf_counter() - t0
        out["inflight"] = inflight
        out["qps_inflight"] = round(B * steps / el2, 1)
        out["frac_end_to_end_inflight"] = round(flops / (el2 / steps) / 1e12 / peak, 4)
        for lj in lanes:
            lj.close()
    idx.close()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--stream", type=int, default=-1, help="-1 auto, 0 slab path, 1 streaming top-K")
    ap.add_argument("--inflight", type=int, default=1, help="also measure with this many batches in flight")
    ap.add_argument("--refine", type=int, default=-1, help="stream_refine: -1 auto, 0 off, 1 the two-level bound")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    f = open(args.out, "a") if args.out else None
    for name in args.cases.split(","):
        res = run_case(name, CASES[name], args.seconds, dev, args.stream, args.inflight, args.refine)
        line = json.dumps(res)
        print(line, flush=True)
        if f:
            f.write(line + "\n")
            f.flush()


if __name__ == "__main__":
    main()
