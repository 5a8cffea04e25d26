"""bench.py — similarity queries/sec + p50 latency on MI355X (BASELINE.json `metric`).

Workload (configs[1]): batch of 256 query embeddings × 25,216 × 384-d item matrix, exact
cosine top-50, one MI355X per rank.  A step = one bb_search over one batch with the item
matrix and the queries already resident in HBM (MFMA scan with fused query normalisation
-> top-K select writing the final lists).  --inflight L (default 3) keeps L batches in
flight per GPU: L index handles on L HIP streams, steps alternating between them, so one
batch's latency-bound select and the scan's last-tile imbalance overlap the next batch's
scan; every step still runs its complete search.  p50_ms is the per-step latency in that
regime, p50_ms_serial the latency of one batch alone.  At 25K items the index does not
shard: with --gpus N every rank serves its own batches against a full
replica ("replicas only", weak scaling, no collective on the data path); value = queries
of all ranks / max-over-ranks wall time.

--workload c4 / c5 runs the large-index configs instead (BASELINE.json configs[3] / [4]):
1M x 768 bf16, B=4096, top-100 / 10M x 384 bf16, B=8192, top-100, the item rows sharded
across the ranks (ShardedIndex: local streaming top-K, one RCCL all-gather of the candidate
keys, bb_finalize merge).  Total items are fixed, so more GPUs means smaller shards
("scaling": "strong"); value = queries answered per second by the whole job.  These are
not the default line (configs[1] is, per BASELINE.json's metric) and run only on request.

Launch: python bench.py [--gpus 1 --steps 500 --warmup 50]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "brickbrain-rec-engine_amd"))

N_ITEMS, DIM, BATCH, TOPK = 25216, 384, 256, 50
HBM_PEAK_GBS = 8000.0
BF16_DENSE_TF = 2500.0   # MI355X dense bf16 MFMA peak (MI355X_MICROARCH.md), no sparsity
F32_DENSE_TF = 157.3


def scan_kernel_info(dtype):
    """(kernel, MFMA instruction peak, MFMA flops executed per algorithmic flop).
    An f32 index runs the split-precision scan: six bf16 MFMAs per fp32 product
    (scan3_kernel.h, bf16x6, fp32-class accuracy) unless BB_NO_SPLIT forces the fp32 MFMA.
    The roofline is priced on ALGORITHMIC flops (2·B·N·d) against the dense MFMA peak of the
    arithmetic type the path computes in (f32: 157.3 TF, bf16: 2.5 PF); the bf16 MFMA issue
    utilisation of the split kernel is reported beside it."""
    if os.environ.get("BB_FORCE_TILED_GEMM"):
        return "gemm_nt_kernel", 1.0
    if dtype == "f32" and not os.environ.get("BB_NO_SPLIT"):
        return "scan3_kernel<48> (bf16x6 split, f32 accumulate)", 6.0
    if dtype == "f32":
        return "scan2_kernel<float,96> (fp32 MFMA)", 1.0
    return "scan2_kernel<uint16_t,48> (bf16 MFMA)", 1.0


def unit_rows_torch(n, d, seed, device):
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.randn((n, d), generator=g, device=device, dtype=torch.float32)
    return x / x.norm(dim=1, keepdim=True)


def load_pmc(dtype):
    """HBM bytes per dominant-kernel launch from the committed rocprofv3 PMC summary."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(dtype, {}).get("gemm")
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except Exception:
        return None


def cpu_baseline(x_np, q_np, k, budget_s=10.0, max_batches=400):
    """The oracle's batched exact cosine top-k (numpy/BLAS) on the host cores."""
    from oracle.restatement import batched_cosine_topk
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:
        cores = os.cpu_count() or 1
    batched_cosine_topk(x_np, q_np[:8], k)  # warm BLAS
    t0 = time.perf_counter()
    nb = 0
    lat = []
    ids0 = None
    while nb < max_batches and time.perf_counter() - t0 < budget_s:
        t1 = time.perf_counter()
        ids, sc = batched_cosine_topk(x_np, q_np, k)
        lat.append(time.perf_counter() - t1)
        if ids0 is None:
            ids0 = ids
        nb += 1
    el = time.perf_counter() - t0
    out = {"value": round(nb * q_np.shape[0] / el, 1), "unit": "queries/s", "cores": int(cores),
           "kind": "port", "p50_ms": round(1e3 * float(np.median(lat)), 3),
           "sample": f"{nb} batches x {q_np.shape[0]} queries x {x_np.shape[0]} x {x_np.shape[1]} fp32 "
                     f"(numpy/BLAS restatement, oracle/restatement.py batched_cosine_topk)"}
    # the reference deployment's setting: one BLAS thread (OMP_NUM_THREADS=1,
    # docker-compose.yml:52-59), a bounded ~5 s sample
    try:
        from threadpoolctl import threadpool_limits
        with threadpool_limits(limits=1, user_api="blas"):
            t0, nb1, lat1 = time.perf_counter(), 0, []
            while nb1 < max_batches and time.perf_counter() - t0 < budget_s / 2:
                t1 = time.perf_counter()
                batched_cosine_topk(x_np, q_np, k)
                lat1.append(time.perf_counter() - t1)
                nb1 += 1
            el1 = time.perf_counter() - t0
        out["value_1_thread"] = round(nb1 * q_np.shape[0] / el1, 1)
        out["p50_ms_1_thread"] = round(1e3 * float(np.median(lat1)), 3)
    except Exception:
        pass
    return out, ids0


SHARDED = {  # BASELINE.json configs[3] / configs[4]
    "c4": dict(n=1_000_000, d=768, B=4096, k=100, cfg="configs[3]: 1M synthetic items x 768-d bf16, batch=4096, "
                                                      "top-100, item rows sharded, RCCL top-K merge"),
    "c5": dict(n=10_000_000, d=384, B=8192, k=100, cfg="configs[4]: 10M synthetic items x 384-d bf16, batch=8192, "
                                                       "top-100, item rows sharded, RCCL top-K merge"),
}


def unit_rows_chunked(n, d, seed, dev, chunk=1 << 20):
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    out = torch.empty((n, d), dtype=torch.float32, device=dev)
    for i in range(0, n, chunk):
        x = torch.randn((min(chunk, n - i), d), generator=g, device=dev)
        out[i:i + x.shape[0]] = x / x.norm(dim=1, keepdim=True)
    return out


def run_sharded(args, rank, world, local, dev):
    """configs[3] / [4]: row-sharded streaming top-K + RCCL key all-gather + finalize."""
    import torch
    import torch.distributed as dist
    from brickrec.distributed import ShardedIndex
    c = SHARDED[args.workload]
    n, d, B, k = c["n"], c["d"], c["B"], c["k"]
    if world == 1 and not dist.is_initialized():  # one rank: a group of one (no collective traffic)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    sh = ShardedIndex(n, dtype="bf16")
    x = unit_rows_chunked(sh.hi - sh.lo, d, 1234 + rank, dev)   # this rank's rows only
    sh.local.upload_items(x, prenormalized=True)
    del x
    torch.cuda.empty_cache()
    q = unit_rows_chunked(B, d, 4321, dev)                      # replicated batch

    def step():
        return sh.search("semantic", k, q_rows=q)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lat = []
    for _ in range(args.steps):
        t1 = time.perf_counter()
        res = step()
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    # dominant kernel (the streaming scan: pilot + stream pass per step), on its own stream
    sh.local.set_profiling(True)
    ps = max(1, min(args.steps, 5))
    for _ in range(ps):
        step()
    torch.cuda.synchronize()
    prof = sh.local.profile()
    sh.local.set_profiling(False)
    n_loc = sh.hi - sh.lo
    gemm_us = 1e3 * prof["gemm"]["ms"] / ps                     # per step (all scan launches)
    flops_loc = 2.0 * B * n_loc * d
    achieved = flops_loc / (gemm_us * 1e-6) / 1e12
    alg_bytes = n_loc * d * 2 + B * d * 4 + B * k * 8
    out = {
        "metric": f"similarity queries/sec + p50 latency, {d}-d x {n:,} items ({c['cfg'].split(':')[0]})",
        "value": round(B * args.steps / el, 1), "unit": "queries/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 4),
        "p50_ms": round(1e3 * float(np.median(lat)), 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic (unit-norm N(0,1) rows, seeds 1234+rank / 4321)",
        "config": {"workload": c["cfg"], "items": n, "items_per_rank": n_loc, "dim": d, "batch": B, "top_k": k,
                   "parallelism": f"rows sharded x{world}" if world > 1 else "single"},
        "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": BF16_DENSE_TF, "unit": "TFLOP/s",
                     "frac": round(achieved / BF16_DENSE_TF, 4), "traffic": None,
                     "kernel": "scan4_kernel (pilot slab + streaming pass), per rank",
                     "kernel_us_per_step": round(gemm_us, 1), "algorithmic_flops_per_step": flops_loc,
                     "algorithmic_bytes_per_step": alg_bytes},
        "kernels_us_per_step": {kk: round(1e3 * v["ms"] / ps, 2) for kk, v in prof.items() if v["launches"]},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        # bounded sample: 64 queries against the first 200K rows, scaled to the full index
        from oracle.restatement import batched_cosine_topk
        ns = 200_000
        xs = sh.local.get_rows(torch.arange(ns, device=dev)).float().cpu().numpy()
        qs = q[:64].cpu().numpy()
        batched_cosine_topk(xs, qs[:4], k)
        t1 = time.perf_counter()
        nb = 0
        while nb < 20 and time.perf_counter() - t1 < 10.0:
            batched_cosine_topk(xs, qs, k)
            nb += 1
        rate = nb * 64 / (time.perf_counter() - t1) * ns / n
        try:
            from threadpoolctl import threadpool_info
            cores = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
        except Exception:
            cores = os.cpu_count() or 1
        out["cpu_baseline"] = {"value": round(rate, 2), "unit": "queries/s", "cores": int(cores),
                               "kind": "port",
                               "sample": f"{nb} batches x 64 queries x {ns} x {d} (numpy/BLAS restatement), "
                                         f"rate scaled by {ns}/{n} items"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--inflight", type=int, default=3, help="batches in flight per GPU (1 = strictly serial)")
    ap.add_argument("--workload", default="c2", choices=["c2", "c4", "c5"],
                    help="c2 = configs[1] (default line); c4 / c5 = the sharded configs[3] / [4]")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if args.workload != "c2":
        return run_sharded(args, rank, world, local, dev)

    import brickrec
    B = args.batch
    x = unit_rows_torch(N_ITEMS, DIM, 1234, dev)              # replica of the item matrix
    # `inflight` batches in flight: each lane is its own index handle (own HIP stream,
    # workspace and 39 MB item copy) serving its own batch; consecutive steps alternate
    # lanes, so one batch's latency-bound select overlaps the next batch's MFMA scan.
    lanes = []
    for j in range(args.inflight):
        q_j = unit_rows_torch(B, DIM, 4321 + rank + 1000 * j, dev)
        idx_j = brickrec.ItemIndex(device=local, dtype=args.dtype)
        idx_j.upload_items(x)
        s_j = torch.cuda.current_stream(dev) if args.inflight == 1 else torch.cuda.Stream(dev)
        run_j, outs_j = idx_j.prepared_search("semantic", TOPK, q_rows=q_j, stream=s_j)
        lanes.append((idx_j, s_j, run_j, outs_j, q_j))
    idx, stream, run, (o_sc, o_ids, o_cnt), q = lanes[0]

    for i in range(args.warmup):
        lanes[i % len(lanes)][2]()
    torch.cuda.synchronize()

    # ---- timed region: K steps, barrier + sync on both sides, max over ranks ----
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        _, s_i, run_i, _, _ = lanes[i % len(lanes)]
        ev[i][0].record(s_i)
        run_i()
        ev[i][1].record(s_i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    lat_ms = np.array([a.elapsed_time(b) for a, b in ev])
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())

    # ---- single-batch latency without other batches in flight (lane 0 alone) ----
    ser = []
    for _ in range(min(args.steps, 200)):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        run()
        b.record(stream)
        ser.append((a, b))
    torch.cuda.synchronize()
    lat_serial = np.array([a.elapsed_time(b) for a, b in ser])

    # ---- per-kernel device time (HIP events on the launch stream), same K steps ----
    idx.set_profiling(True)
    for _ in range(args.steps):
        run()
    prof = idx.profile()
    idx.set_profiling(False)
    g = prof["gemm"]
    gemm_us = 1e3 * g["ms"] / max(g["launches"], 1)
    flops = 2.0 * B * N_ITEMS * DIM
    es = 4 if args.dtype == "f32" else 2
    alg_bytes = N_ITEMS * DIM * es + B * DIM * 4 + B * TOPK * 8    # items + queries + top-K out
    kname, mfma_per_flop = scan_kernel_info(args.dtype)
    bound, unit = "mfma", "TFLOP/s"
    peak = F32_DENSE_TF if args.dtype == "f32" else BF16_DENSE_TF
    achieved = flops / (gemm_us * 1e-6) / 1e12  # algorithmic flops per launch / launch time
    mfma_issue_tflops = achieved * mfma_per_flop  # bf16 MFMA flops the kernel actually issues
    hbm = load_pmc(args.dtype)

    # ---- MALL-cold latency (256 MiB Infinity Cache flushed before each step) ----
    flush = torch.empty(640 << 20, dtype=torch.uint8, device=dev)
    cold = []
    for i in range(20):
        with torch.cuda.stream(stream):
            flush.fill_(i & 0xFF)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        run()
        b.record(stream)
        torch.cuda.synchronize()
        cold.append(a.elapsed_time(b))
    del flush

    out = {
        "metric": "similarity queries/sec + p50 latency, 384-d x 25,216 items (configs[1])",
        "value": round(world * B * args.steps / el, 1),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * el / args.steps, 4),
        "p50_ms": round(float(np.median(lat_ms)), 4),
        "p50_ms_serial": round(float(np.median(lat_serial)), 4),
        "p50_ms_mall_cold": round(float(np.median(cold)), 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (unit-norm N(0,1) rows, seeds 1234 / 4321+rank)",
        "config": {"workload": "configs[1]: batch=256 queries x 25,216 x 384-d items, cosine top-50",
                   "items": N_ITEMS, "dim": DIM, "batch": B, "top_k": TOPK,
                   "parallelism": f"replicas x{world}" if world > 1 else "single",
                   "inflight_batches": args.inflight},
        "roofline": {"bound": bound, "achieved": round(achieved, 2), "peak": peak, "unit": unit,
                     "frac": round(achieved / peak, 4), "traffic": hbm,
                     "kernel": kname, "kernel_us": round(gemm_us, 3),
                     "mfma_flops_per_algorithmic_flop": mfma_per_flop,
                     "bf16_mfma_issue_tflops": round(mfma_issue_tflops, 2),
                     "bf16_mfma_issue_frac": round(mfma_issue_tflops / BF16_DENSE_TF, 4),
                     "algorithmic_flops_per_launch": flops, "algorithmic_bytes_per_launch": alg_bytes,
                     "hbm_frac_at_alg_bytes": round(alg_bytes / (gemm_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)},
        "kernels_us_per_step": {k: round(1e3 * v["ms"] / max(args.steps, 1), 3) for k, v in prof.items()
                                if v["launches"]},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        x_np = x.cpu().numpy()
        q_np = q.cpu().numpy()
        cb, ids0 = cpu_baseline(x_np, q_np, TOPK)
        gpu_ids = o_ids.cpu().numpy()
        same = float(np.mean([set(gpu_ids[i]) == set(ids0[i]) for i in range(B)]))
        cb["topk_set_agreement_with_gpu"] = round(same, 4)
        out["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
