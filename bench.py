"""bench.py — similarity queries/sec + p50 latency on MI355X (BASELINE.json `metric`).

Workload (configs[1], the default line): batch of 256 query embeddings × 25,216 × 384-d item
matrix, exact cosine top-50, one MI355X per rank.  A step = one bb_search over one batch
with the item matrix and the queries already resident in HBM.  --inflight L (default 3)
keeps L batches in flight per GPU: L index handles on L HIP streams, steps alternating
between them, so one batch's latency-bound select overlaps the next batch's scan; every
step still runs its complete search.  p50_ms is the per-step latency in that regime,
p50_ms_serial the latency of one batch alone.  At 25K items the index does not shard
(SURVEY.md §8e): with --gpus N every rank serves its own batches against a full replica
("replicas only", weak scaling, no collective on the data path); value = queries of all
ranks / max-over-ranks wall time.

Other workloads (run on request, not the default line):
  --workload c3   configs[2]: hybrid (liked-set content + CF r=50) + the constraint mask
                  (num_parts <= 800 AND year >= 2015) + rated exclusions, B=1024, top-50, f32
  --workload c4   configs[3]: 1M x 768 bf16, B=4096, top-100, rows sharded over the ranks
  --workload c5   configs[4]: 10M x 384 bf16, B=8192, top-100, rows sharded over the ranks
The sharded workloads (ShardedIndex: local streaming top-K, one RCCL all-gather of the
candidate keys, bb_finalize merge) fix the total items, so more GPUs means smaller shards
("scaling": "strong").

Roofline (dominant kernel = the scan launches of a step, HIP events on the library's launch
stream; see roofline()): the binding side follows SURVEY.md §8(d), max(issued MFMA flops /
MFMA peak, algorithmic bytes / HBM peak).  The f32 index runs the exact re-rank path (a
one-product f16 MFMA scan over the index's f16 copy, then the list select rescores the
candidates within its proven error bound from the f32 rows), so at configs[1] the algorithmic model binds on HBM (39.2 MB
of f32 rows vs 4.96 GFLOP).  `f32_equivalent` prices the algorithmic flops against the f32
MFMA peak (157.3 TF).

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
BF16_DENSE_TF = 2500.0   # MI355X dense bf16 / f16 MFMA peak (MI355X_MICROARCH.md), no sparsity
F32_DENSE_TF = 157.3


def scan_kernel_info(dtype, width, batch):
    """(kernel, MFMA flops executed per algorithmic flop) of the scan that runs for an index
    of this dtype and padded width on a one-slab search.  An f32 index runs the exact
    re-rank path: a one-product f16 MFMA scan (scan2 for up to 256 queries, scan4 above)
    gives approximate scores within a proven bound and keeps bounded per-lane candidate lists,
    and select_list_kernel rescores the candidates within the bound from the f32 rows
    (BB_AB=1 BB_NO_RR forces the older split-precision scan3, six bf16 products per fp32
    product).  A bf16 index runs scan2 / scan4 directly."""
    ab = os.environ.get("BB_AB")   # A/B switches are honoured only with BB_AB set (csrc/common.h ab_env)
    if ab and os.environ.get("BB_FORCE_TILED_GEMM"):
        return "gemm_nt_kernel", 1.0
    kern = "scan4_kernel" if batch > 256 else "scan2_kernel"
    if dtype == "f32" and ab and os.environ.get("BB_NO_RR") and not os.environ.get("BB_NO_SPLIT"):
        return f"scan3_kernel<{width * 2 // 16}> (bf16x6 split, f32 accumulate)", 6.0
    if dtype == "f32" and ab and os.environ.get("BB_NO_RR"):
        return "scan2_kernel<float> (fp32 MFMA)", 1.0
    if dtype == "f32":
        return (f"{kern}<uint16_t,{width * 2 // 16},list|f16> (one-product f16 approximate scan, bounded per-lane "
                f"candidate lists in the epilogue, no score image; exact f32 re-rank of the candidates in "
                f"select_list_kernel)"), 1.0
    return f"{kern}<uint16_t,{width * 2 // 16}> (bf16 MFMA)", 1.0


def roofline(flops_alg, bytes_alg, kernel_us, dtype, kname, mfma_per_flop, traffic, mfma16=False):
    """Roofline object of one kernel.  The binding ceiling follows SURVEY.md §8(d):
    max(issued MFMA flops / MFMA peak, algorithmic bytes / HBM peak).  `achieved` is the
    binding side's rate: issued MFMA TFLOP/s (algorithmic flops × MFMA flops per algorithmic
    flop) against the dense peak of the issued instruction, or algorithmic GB/s against HBM;
    the other side is reported beside it."""
    t = kernel_us * 1e-6
    alg_tf = flops_alg / t / 1e12
    issued = alg_tf * mfma_per_flop
    # mfma16: the search's flops run on a 16-bit MFMA (the f32 index's one-product f16 scan),
    # so every family of that search is priced against the 16-bit dense peak
    peak_tf = (BF16_DENSE_TF if (mfma16 or dtype == "bf16" or mfma_per_flop > 1 or "bf16" in kname or "f16" in kname)
               else F32_DENSE_TF)
    gbs = bytes_alg / t / 1e9
    t_mfma = flops_alg * mfma_per_flop / (peak_tf * 1e12)
    t_hbm = bytes_alg / (HBM_PEAK_GBS * 1e9)
    if t_hbm > t_mfma:
        out = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic}
    else:
        out = {"bound": "mfma", "achieved": round(issued, 2), "peak": peak_tf, "unit": "TFLOP/s",
               "frac": round(issued / peak_tf, 4), "traffic": traffic}
    out.update({"kernel": kname, "kernel_us": round(kernel_us, 3),
                "ideal_us": {"mfma": round(1e6 * t_mfma, 3), "hbm": round(1e6 * t_hbm, 3)},
                "mfma_issued_tflops": round(issued, 2), "mfma_frac": round(issued / peak_tf, 4),
                "mfma_peak": peak_tf, "mfma_flops_per_algorithmic_flop": mfma_per_flop,
                "algorithmic_tflops": round(alg_tf, 2), "hbm_gbs_at_alg_bytes": round(gbs, 1),
                "hbm_frac_at_alg_bytes": round(gbs / HBM_PEAK_GBS, 4),
                "algorithmic_flops_per_launch": flops_alg, "algorithmic_bytes_per_launch": bytes_alg})
    if dtype == "f32":
        out["f32_equivalent"] = {"achieved": round(alg_tf, 2), "peak": F32_DENSE_TF,
                                 "frac": round(alg_tf / F32_DENSE_TF, 4)}
    return out


def family_kernels(workload, dtype, B, scan_name):
    """Kernel behind each profiling family of bb_get_profile (HIP events on the launch stream)."""
    if workload == "c2" and dtype == "f32" and B <= 16:
        return {"gemm": "sq_scan_kernel (approximate f16 MFMA pass, small batch)", "select": "sq_merge_kernel"}
    if workload == "c3":
        return {"pack": "compact_kernel (constraint-first packing of the allowed rows + both sides' query prep)",
                "prep": "prep2_kernel", "gemm": scan_name, "select": "select_list_dual_kernel",
                "finalize": "finalize1_mid_kernel (two waves per row: side lists of <= 128 keys)"}
    return {"prep": "prep_kernel", "gemm": scan_name,
            "select": "select_list_kernel" if dtype == "f32" else "select_kernel", "rerank": "rerank_kernel",
            "finalize": "finalize1_kernel"}


def scan_read_roofline(B, d, scan_us, n=N_ITEMS, cus=256):
    """the f32 index's scan never reads the f32 rows §8(d) prices — it reads
    their f16 re-rank copy and f16 query operands.  Two more honest denominators for the scan:
    (1) the bytes it must read (f16 rows + f16 queries) against HBM peak; (2) the per-CU
    operand-delivery floor: a B × n score block split over P CUs needs at least 2·√(B·n/P)·d·2
    bytes delivered to each CU (square tiles), at the per-CU rates tools/percu_probe measured
    (profiles/r05_percu_probe.jsonl, 256 KiB per CU: 66.9 GB/s from a shared, L2-resident
    region; 25.3 GB/s from regions each XCD must fetch from the Infinity Cache)."""
    must = n * d * 2 + B * d * 2
    t = scan_us * 1e-6
    per_cu = 2.0 * (B * n / cus) ** 0.5 * d * 2
    rates = {"l2_shared": 66.9e9, "infinity_cache": 25.3e9}
    floors = {k: per_cu / r * 1e6 for k, r in rates.items()}
    return {"must_read_bytes": must, "achieved_gbs": round(must / t / 1e9, 1),
            "frac_hbm_peak": round(must / t / 1e9 / HBM_PEAK_GBS, 4),
            "operand_bytes_per_cu": round(per_cu), "delivery_floor_us": {k: round(v, 2) for k, v in floors.items()},
            "frac_of_delivery_floor": {k: round(v / scan_us, 4) for k, v in floors.items()},
            "source": "profiles/r05_percu_probe.jsonl (tools/percu_probe.hip)"}


def dominant_roofline(fam_us, names, flops, alg_bytes, step_us, dtype, scan_mpf, pmc_key, mfma16=False):
    """roofline object for the kernel family that takes the most device time per step (HIP
    events, bb_get_profile), with SURVEY.md §8(d)'s algorithmic work of one search priced
    against that kernel's time; `step` prices the same work against the whole step (wall time
    per step of the timed window), `scan` reports the scan launch's own MFMA / HBM rates."""
    dom = max(fam_us, key=fam_us.get)
    kname = names.get(dom, dom)
    mpf = scan_mpf if dom == "gemm" else 1.0
    out = roofline(flops, alg_bytes, fam_us[dom], dtype, kname, mpf, load_pmc(pmc_key, dom), mfma16)
    out["family"] = dom
    out["step"] = {"us": round(step_us, 3), "achieved_gbs": round(alg_bytes / (step_us * 1e-6) / 1e9, 1),
                   "frac": round(alg_bytes / (step_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                   "note": "algorithmic bytes of one search / wall time per step of the timed window"}
    if "gemm" in fam_us:
        sc = roofline(flops, alg_bytes, fam_us["gemm"], dtype, names.get("gemm", "gemm"), scan_mpf,
                      load_pmc(pmc_key, "gemm"), mfma16)
        out["scan"] = {k: sc[k] for k in ("kernel", "kernel_us", "mfma_issued_tflops", "mfma_frac",
                                          "hbm_frac_at_alg_bytes", "traffic")}
    return out


def unit_rows_torch(n, d, seed, device, chunk=1 << 20):
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.empty((n, d), dtype=torch.float32, device=device)
    for i in range(0, n, chunk):
        x = torch.randn((min(chunk, n - i), d), generator=g, device=device, dtype=torch.float32)
        out[i:i + x.shape[0]] = x / x.norm(dim=1, keepdim=True)
    return out


def load_pmc(key, family="gemm"):
    """HBM bytes per step of one kernel family from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, tools/pmc_traffic.py), or None when not collected."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(key, {}).get(family)
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except Exception:
        return None


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:
        return os.cpu_count() or 1


def _time_cpu(fn, budget_s, max_calls):
    fn()  # warm
    lat = []
    t0 = time.perf_counter()
    while len(lat) < max_calls and time.perf_counter() - t0 < budget_s:
        t1 = time.perf_counter()
        fn()
        lat.append(time.perf_counter() - t1)
    return len(lat), time.perf_counter() - t0, lat


def cpu_baseline(x_np, q_np, k, budget_s=8.0, sweep_s=2.0):
    """The oracle's batched exact cosine top-k (numpy/BLAS: the sequential-scan semantics of
    pgvector / FAISS IndexFlat) on the host cores, timed — never extrapolated.  `value` is the
    workload's own batch on all BLAS threads; `sweep` times B ∈ {1 (top-10, configs[0]), 256,
    1024, 4096} on all threads and on one thread (the reference deployment's
    OMP_NUM_THREADS=1, docker-compose.yml:52-59)."""
    from oracle.restatement import batched_cosine_topk
    cores = _blas_threads()
    B = q_np.shape[0]
    ids0 = batched_cosine_topk(x_np, q_np, k)[0]
    nb, el, lat = _time_cpu(lambda: batched_cosine_topk(x_np, q_np, k), budget_s, 400)
    out = {"value": round(nb * B / el, 1), "unit": "queries/s", "cores": int(cores), "kind": "port",
           "rank": 0,
           "p50_ms": round(1e3 * float(np.median(lat)), 3),
           "sample": f"{nb} batches x {B} queries x {x_np.shape[0]} x {x_np.shape[1]} fp32 (numpy/BLAS restatement, "
                     f"oracle/restatement.py batched_cosine_topk), timed"}
    rng = np.random.default_rng(99)
    qs = rng.standard_normal((4096, x_np.shape[1])).astype(np.float32)
    sweep = []
    try:
        from threadpoolctl import threadpool_limits
    except Exception:
        threadpool_limits = None
    for threads in ((cores, 1) if sweep_s > 0 else ()):
        for b, kk in ((1, 10), (256, 50), (1024, 50), (4096, 50)):
            qb = qs[:b]

            def call():
                batched_cosine_topk(x_np, qb, kk)
            if threads == 1 and threadpool_limits is not None:
                with threadpool_limits(limits=1, user_api="blas"):
                    n_, el_, lat_ = _time_cpu(call, sweep_s, 2000)
            elif threads == 1:
                continue
            else:
                n_, el_, lat_ = _time_cpu(call, sweep_s, 2000)
            sweep.append({"B": b, "k": kk, "threads": int(threads), "queries_per_s": round(n_ * b / el_, 1),
                          "p50_ms": round(1e3 * float(np.median(lat_)), 3), "calls": n_})
    out["sweep"] = sweep
    one = [s for s in sweep if s["threads"] == 1 and s["B"] == B]
    if one:
        out["value_1_thread"] = one[0]["queries_per_s"]
        out["p50_ms_1_thread"] = one[0]["p50_ms"]
    return out, ids0


def cpu_baseline_hybrid(x_np, f_np, mask, liked, rated, u, k, budget_s=10.0, n_sample=64):
    """configs[2] on the host: the oracle's HybridRecommender scoring path
    (recommendation_system.py:612-677) per query — liked-set cosine over every item with the
    rank-0 drop and the mask (:194-249, top 2k), CF u·Fᵀ with rated items and the mask
    excluded (:411-483, top 2k), union blend 0.4/0.6 (:789-843) — the cosine and CF products
    batched through numpy/BLAS, timed on a bounded sample of the workload's own queries, on
    all BLAS threads and on one (the reference deployment's OMP_NUM_THREADS=1)."""
    from oracle import restatement as R
    xn = R.normalize_rows(x_np)
    nq = min(n_sample, len(liked))

    def run(nq_):
        sim = xn[liked[:nq_]] @ xn.T                       # cosine_similarity(x_t, X), batched
        fs = u[:nq_] @ f_np.T                              # user_factors[u] · item_factors.T
        res = []
        for b in range(nq_):
            drop = R.rank0(sim[b])
            okc = mask.copy()
            okc[drop] = False
            ci, cs = R.topk_indices(sim[b], 2 * k, okc)
            fi, fsc = R.topk_indices(fs[b], 2 * k, mask & ~rated[b])
            res.append(R.union_blend(ci, cs, fi, fsc, 0.4, 0.6, k)[0])
        return res
    ids0 = run(nq)
    out = {"unit": "queries/s", "kind": "port", "cores": int(_blas_threads()),
           "sample": f"{nq} configs[2] queries per call (the bench's own liked sets, users, mask and rated items) "
                     f"x {x_np.shape[0]} x {x_np.shape[1]} fp32 + r={f_np.shape[1]} CF: oracle/restatement.py "
                     f"similar_sets + cf_topk + union_blend semantics, numpy/BLAS, timed"}
    n_, el, lat = _time_cpu(lambda: run(nq), budget_s, 200)
    out["value"] = round(n_ * nq / el, 1)
    out["p50_ms_per_call"] = round(1e3 * float(np.median(lat)), 2)
    try:
        from threadpoolctl import threadpool_limits
        with threadpool_limits(limits=1, user_api="blas"):
            n1, el1, _ = _time_cpu(lambda: run(nq), budget_s / 2, 100)
        out["value_1_thread"] = round(n1 * nq / el1, 1)
    except Exception:
        pass
    return out, ids0


SHARDED = {  # BASELINE.json configs[3] / configs[4]
    "c4": dict(n=1_000_000, d=768, B=4096, k=100, cfg="configs[3]: 1M synthetic items x 768-d bf16, batch=4096, "
                                                      "top-100, item rows sharded, RCCL top-K merge"),
    "c5": dict(n=10_000_000, d=384, B=8192, k=100, cfg="configs[4]: 10M synthetic items x 384-d bf16, batch=8192, "
                                                       "top-100, item rows sharded, RCCL top-K merge"),
}


def cpu_full_scan(get_chunk, n, q_np, k, budget_s=12.0, chunk=1 << 19):
    """Timed CPU baseline over the WHOLE index (no extrapolation): the numpy/BLAS restatement
    scanning the rows in chunks (a sequential scan, as pgvector / FAISS IndexFlat do) for a
    bounded query sample, keeping the running exact top-k."""
    from oracle.restatement import normalize_rows
    qn = normalize_rows(q_np)
    rows = [get_chunk(c0, min(n, c0 + chunk)) for c0 in range(0, n, chunk)]   # host copy, untimed

    def scan(nq):
        best_s = np.full((nq, k), -np.inf, np.float32)
        best_i = np.zeros((nq, k), np.int64)
        for ci, xr in enumerate(rows):
            s = qn[:nq] @ xr.T
            part = np.argpartition(-s, k - 1, axis=1)[:, :k]
            cs = np.concatenate([best_s, np.take_along_axis(s, part, 1)], 1)
            cid = np.concatenate([best_i, part + ci * chunk], 1)
            o = np.argpartition(-cs, k - 1, axis=1)[:, :k]
            best_s, best_i = np.take_along_axis(cs, o, 1), np.take_along_axis(cid, o, 1)
        return best_i
    t0 = time.perf_counter()
    scan(1)
    t_one = time.perf_counter() - t0
    nq = int(max(1, min(q_np.shape[0], 64)))
    t0 = time.perf_counter()
    calls = 0
    while calls < 3 and time.perf_counter() - t0 < budget_s:
        scan(nq)
        calls += 1
    el = time.perf_counter() - t0
    return {"value": round(calls * nq / el, 2), "unit": "queries/s", "cores": int(_blas_threads()), "kind": "port",
            "p50_ms_B1": round(1e3 * t_one, 2),
            "sample": f"{calls} batches x {nq} queries over all {n} rows x {q_np.shape[1]} (bf16 rows widened to "
                      f"f32; numpy/BLAS chunked sequential scan), timed over the full index"}


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
    x = unit_rows_torch(sh.hi - sh.lo, d, 1234 + rank, dev)   # this rank's rows only
    sh.upload_items(x, prenormalized=True)
    del x
    torch.cuda.empty_cache()
    q = unit_rows_torch(B, d, 4321, dev)                      # replicated batch

    def step():
        return sh.search("semantic", k, q_rows=q, pipeline=args.pipeline)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lat = []
    for _ in range(args.steps):
        t1 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    # dominant kernel (the streaming scan: pilot + stream passes per step), on its own stream
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
    alg_bytes = n_loc * d * 2 + B * d * 4 + B * k * 8
    out = {
        "metric": f"similarity queries/sec + p50 latency, {d}-d x {n:,} items ({c['cfg'].split(':')[0]})",
        "value": round(B * args.steps / el, 1), "unit": "queries/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 4),
        "p50_ms": round(1e3 * float(np.median(lat)), 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic (unit-norm N(0,1) rows, seeds 1234+rank / 4321)",
        "config": {"workload": c["cfg"], "items": n, "items_per_rank": n_loc, "dim": d, "batch": B, "top_k": k,
                   "parallelism": f"rows sharded x{world}" if world > 1 else "single"},
        "roofline": roofline(flops_loc, alg_bytes, gemm_us, "bf16",
                             "scan4_kernel<uint16_t> bf16 (pilot slab + streaming passes), per rank, per step", 1.0,
                             load_pmc(args.workload)),
        "kernels_us_per_step": {kk: round(1e3 * v["ms"] / ps, 2) for kk, v in prof.items() if v["launches"]},
        "cpu_baseline": None,
    }
    if rank == 0 and not args.no_cpu:
        # the CPU baseline scans the WHOLE index at every N: rank 0's own
        # stored rows, and every other rank's shard regenerated as that rank made it (same
        # seed, rounded to bf16 as stored)
        from brickrec.distributed import shard_bounds
        def shard_rows(r):
            lo_r, hi_r = shard_bounds(n, world, r)
            if r == rank:
                return lambda a, b: sh.local.get_rows(torch.arange(a - lo_r, b - lo_r, device=dev)).float().cpu().numpy()
            def rows(a, b):   # lazily, one regenerated shard held at a time
                if cache.get("r") != r:
                    cache.clear()
                    cache["x"] = unit_rows_torch(hi_r - lo_r, d, 1234 + r, dev).to(torch.bfloat16).float().cpu().numpy()
                    cache["r"] = r
                return cache["x"][a - lo_r:b - lo_r]
            return rows
        cache = {}
        owners = [(shard_bounds(n, world, r), shard_rows(r)) for r in range(world)]

        def get_chunk(a, b):   # global rows [a, b), possibly spanning shards
            parts = [f(max(a, lo_r), min(b, hi_r)) for (lo_r, hi_r), f in owners if max(a, lo_r) < min(b, hi_r)]
            return np.concatenate(parts, 0)
        out["cpu_baseline"] = cpu_full_scan(get_chunk, n, q[:64].cpu().numpy(), k)
        del owners, cache
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def make_base(brickrec, workload, x, local, dtype, extra):
    """The resident index of this GPU: one copy of the rows (and CF factors / attributes)."""
    idx = brickrec.ItemIndex(device=local, dtype=dtype)
    idx.upload_items(x)
    if workload == "c3":
        idx.upload_cf(extra["f"])
        idx.upload_attrs(extra["parts"], extra["year"], extra["theme"])
    return idx


def make_lane(brickrec, workload, base, B, local, dev, rank, j, inflight, extra):
    """One in-flight lane: a view of the resident index (own HIP stream + workspace, shared rows,
    bb_create_view) and its own batch."""
    import torch
    idx = base.view()
    s = torch.cuda.current_stream(dev) if inflight == 1 else torch.cuda.Stream(dev)
    if workload == "c3":
        mask = idx.eval_mask(brickrec.Predicate(parts_max=800, year_min=2015))
        rng = np.random.default_rng(7000 + rank + 10 * j)
        liked = rng.choice(N_ITEMS, B, replace=False)
        rated = np.zeros((B, N_ITEMS), bool)
        for b in range(B):
            rated[b, rng.choice(N_ITEMS, int(rng.integers(10, 31)), replace=False)] = True
        u = rng.normal(0.0, 0.1, (B, extra["f"].shape[1])).astype(np.float32)
        mw = torch.from_numpy(brickrec.bits_from_bool(mask).view(np.int32)).to(dev)
        ew = torch.from_numpy(brickrec.bits_from_bool(rated).view(np.int32)).to(dev)
        # mask_count: the allowed rows' count (the reference's len(valid_set_nums), :634) lets
        # the search pack them first (constraint-first, BB_OPT_PREFILTER) — computed here once
        # per lane with the mask, as the serving path computes it with the constraint
        kw = dict(q_items=torch.from_numpy(liked).to(dev), q_cf=torch.from_numpy(u).to(dev), mask=mw, excl=ew,
                  stream=s, mask_count=int(np.count_nonzero(mask)))
        run, outs = idx.prepared_search("hybrid", TOPK, **kw)
        # the profiled runs go through bb_search on the lane's own handle (a plan replays on its
        # private view, which the lane's profiler does not see): the same kernels and arguments
        run.prof_run = idx.prepared_search("hybrid", TOPK, plan=False, **kw)[0]
        return idx, s, run, outs, {"liked": liked, "rated": rated, "u": u, "mask": np.asarray(mask, bool)}
    q = unit_rows_torch(B, DIM, 4321 + rank + 1000 * j, dev)
    run, outs = idx.prepared_search("semantic", TOPK, q_rows=q, stream=s)
    run.prof_run = idx.prepared_search("semantic", TOPK, q_rows=q, stream=s, plan=False)[0]
    return idx, s, run, outs, q


def gpu_batch_sweep(brickrec, base, local, dev, seconds=0.5):
    """GPU q/s (3 in flight) and serial p50 at B ∈ {1 (top-10), 16, 64, 256, 1024, 4096}:
    the north_star's batch axis at 25K items."""
    import torch
    res = []
    for b, kk in ((1, 10), (16, 50), (64, 50), (256, 50), (1024, 50), (4096, 50)):
        lanes = []
        for j in range(3):
            idx = base.view()
            q = unit_rows_torch(b, DIM, 555 + j, dev)
            s = torch.cuda.Stream(dev)
            run, _ = idx.prepared_search("semantic", kk, q_rows=q, stream=s)
            lanes.append((idx, s, run, q))
        for i in range(30):
            lanes[i % 3][2]()
        torch.cuda.synchronize()
        steps = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for _ in range(30):
                lanes[steps % 3][2]()
                steps += 1
            torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ser = []
        idx0, s0, run0, _ = lanes[0]
        for _ in range(100):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s0)
            run0()
            e.record(s0)
            ser.append((a, e))
        torch.cuda.synchronize()
        res.append({"B": b, "k": kk, "queries_per_s_inflight3": round(steps * b / el, 1),
                    "p50_ms_serial": round(float(np.median([a.elapsed_time(e) for a, e in ser])), 4)})
        for ln in lanes:
            ln[0].close()
    return res


def request_latency(brickrec, x, dev, reps=100):
    """Serial p50 of single requests in the reference's own shapes (one call at a time on an
    idle stream, HIP events): get_similar_sets top-10 (recommendation_system.py:194-249), the
    pgvector retriever k=20 (lego_nlp_recommeder.py:305, 1394), CF top-20 of one user with
    rated items excluded (:411-483), and HybridRecommender.get_recommendations top-10 with
    the configs[2] mask and rated exclusions (:612-677) — f32 index with r=50 CF factors."""
    import torch
    rng = np.random.default_rng(77)
    f = rng.normal(0.0, 0.1, (N_ITEMS, 50)).astype(np.float32)
    idx = brickrec.ItemIndex(device=dev.index, dtype="f32")
    idx.upload_items(x)
    idx.upload_cf(f)
    parts = rng.integers(1, 6000, N_ITEMS).astype(np.int32)
    year = rng.integers(1949, 2025, N_ITEMS).astype(np.int16)
    idx.upload_attrs(parts, year, rng.integers(0, 400, N_ITEMS).astype(np.int32))
    mask = torch.from_numpy(brickrec.bits_from_bool(idx.eval_mask(brickrec.Predicate(parts_max=800, year_min=2015)))
                            .view(np.int32)).to(dev)
    rated = np.zeros((1, N_ITEMS), bool)
    rated[0, rng.choice(N_ITEMS, 20, replace=False)] = True
    excl = torch.from_numpy(brickrec.bits_from_bool(rated).view(np.int32)).to(dev)
    liked = torch.tensor([int(rng.integers(N_ITEMS))], device=dev)
    u = torch.from_numpy(rng.normal(0.0, 0.1, (1, 50)).astype(np.float32)).to(dev)
    q = unit_rows_torch(1, DIM, 991, dev)
    s = torch.cuda.Stream(dev)
    cases = {"similar_k10": dict(mode="similar", k=10, q_items=liked),
             "retriever_k20": dict(mode="semantic", k=20, q_rows=q),
             "cf_k20_rated": dict(mode="cf", k=20, q_cf=u, excl=excl),
             "hybrid_k10_mask_rated": dict(mode="hybrid", k=10, q_items=liked, q_cf=u, mask=mask, excl=excl)}
    out = {}
    for name, c in cases.items():
        c = dict(c)
        run, _ = idx.prepared_search(c.pop("mode"), c.pop("k"), stream=s, **c)
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        ev = []
        for _ in range(reps):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            run()
            e.record(s)
            ev.append((a, e))
        torch.cuda.synchronize()
        out[name] = round(float(np.median([a.elapsed_time(e) for a, e in ev])), 4)
    idx.close()
    return {"p50_ms_serial": out, "note": "B=1 requests on an idle stream, 25,216 x 384 f32 + r=50 CF"}


def launch_ranks(args):
    """`--gpus N` without a launcher: start the N rank processes (torch.distributed.run on
    127.0.0.1, one rank per GPU) as a child before this process touches any GPU, and return
    its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def dry_run(args):
    """Device-free rehearsal (tests/test_bench_launcher.py): the ranks join a gloo group, run
    the timed region's barriers and max-over-ranks reduction around a no-op step, and rank 0
    times the CPU baseline on a small sample and prints the line.  Nothing is measured on a
    GPU: value is null."""
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    sharded = args.workload in SHARDED
    out = {"metric": "similarity queries/sec + p50 latency, 384-d x 25,216 items (configs[1])", "value": None,
           "unit": "queries/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "dry_run": True,
           "ms_per_step": None, "higher_is_better": True, "scaling": "strong" if sharded else "weak",
           "vs_baseline": None, "dtype": args.dtype, "data": "synthetic", "max_rank_s": float(t.item()),
           "config": {"workload": f"dry run (no device) of {args.workload}",
                      "parallelism": (f"rows sharded x{world}" if sharded else f"replicas x{world}") if world > 1
                      else "single"},
           "roofline": None, "cpu_baseline": None}
    if rank == 0 and not args.no_cpu:
        from oracle.restatement import unit_rows
        if sharded:   # the sharded CPU leg (cpu_full_scan over every rank's rows), on a small index
            from brickrec.distributed import shard_bounds
            c = SHARDED[args.workload]
            n_dry = 8192
            shards = [unit_rows(hi - lo, c["d"], 1234 + r) for r, (lo, hi) in
                      enumerate(shard_bounds(n_dry, world, r) for r in range(world))]
            full = np.concatenate(shards, 0)
            out["cpu_baseline"] = cpu_full_scan(lambda a, b: full[a:b], n_dry, unit_rows(64, c["d"], 4321), c["k"],
                                                budget_s=args.cpu_budget, chunk=4096)
            out["cpu_baseline"]["sample"] += f" (dry run: {n_dry:,} rows in {world} shards)"
        else:
            x_np = unit_rows(4096, DIM, 1234)
            q_np = unit_rows(BATCH, DIM, 4321)
            out["cpu_baseline"], _ = cpu_baseline(x_np, q_np, TOPK, budget_s=args.cpu_budget, sweep_s=0.0)
            out["cpu_baseline"]["sample"] += " (dry run: 4,096 rows)"
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-sweep", action="store_true", help="skip the GPU batch sweep")
    ap.add_argument("--inflight", type=int, default=3, help="batches in flight per GPU (1 = strictly serial)")
    ap.add_argument("--lane-copies", action="store_true", help="one uploaded copy of the rows per in-flight lane")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="c2 = configs[1] (default line); c3 = configs[2] hybrid; c4 / c5 = the sharded configs[3] / [4]")
    ap.add_argument("--dry-run", action="store_true",
                    help="device-free rehearsal of the launcher and the reporting path (gloo ranks, no GPU)")
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds of CPU-baseline timing")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="sharded workloads: query chunks whose key all-gathers overlap the next chunk's search")
    ap.add_argument("--mall-flush", action="store_true",
                    help="flush the 256 MiB Infinity Cache before every timed step (cold-MALL profiling runs; "
                         "use with --inflight 1 under rocprofv3)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args)
    if args.dry_run:
        return dry_run(args)

    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)   # RCCL
        world = dist.get_world_size()                    # n_gpus = the ranks that joined
    if args.workload in SHARDED:
        return run_sharded(args, rank, world, local, dev)

    import brickrec
    hybrid = args.workload == "c3"
    B = args.batch or (1024 if hybrid else BATCH)
    x = unit_rows_torch(N_ITEMS, DIM, 1234, dev)              # replica of the item matrix
    extra = {}
    if hybrid:
        rng = np.random.default_rng(2024)
        extra = {"f": rng.normal(0.0, 0.1, (N_ITEMS, 50)).astype(np.float32),
                 "parts": rng.integers(1, 6000, N_ITEMS).astype(np.int32),
                 "year": rng.integers(1949, 2025, N_ITEMS).astype(np.int16),
                 "theme": rng.integers(0, 400, N_ITEMS).astype(np.int32)}
    # `inflight` batches in flight: each lane is a view of one resident index (own HIP
    # stream and workspace, the rows shared) serving its own batch; consecutive steps
    # alternate lanes, so one batch's latency-bound select overlaps the next batch's scan.
    base = make_base(brickrec, args.workload, x, local, args.dtype, extra)
    # (--lane-copies: every lane uploads its own copy of the rows — the round-1 scheme, A/B runs)
    lanes = [make_lane(brickrec, args.workload,
                       make_base(brickrec, args.workload, x, local, args.dtype, extra) if args.lane_copies else base,
                       B, local, dev, rank, j, args.inflight, extra)
             for j in range(args.inflight)]
    idx, stream, run, (o_sc, o_ids, o_cnt), q = lanes[0]

    # ---- single-batch latency without other batches in flight (lane 0 alone, 200 batches) ----
    # Measured before the warmup steps, so the timed window opens on a GPU that has been serving
    # (a 20-step window otherwise starts on the clocks of the idle before it).
    ser = []
    for _ in range(200):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        run()
        b.record(stream)
        ser.append((a, b))
    torch.cuda.synchronize()
    lat_serial = np.array([a.elapsed_time(b) for a, b in ser])
    for i in range(args.warmup):
        lanes[i % len(lanes)][2]()
    torch.cuda.synchronize()

    # ---- timed region: K steps, barrier + sync on both sides, max over ranks ----
    # (nothing but the steps inside: a pair of per-step events costs the host about as much
    # as a plan launch, and at 20 steps the host would pace the pipeline fill)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    flush = torch.empty(640 << 20, dtype=torch.uint8, device=dev) if args.mall_flush else None
    t0 = time.perf_counter()
    for i in range(args.steps):
        if flush is not None:   # (profiling runs only: the fill is inside the window)
            with torch.cuda.stream(lanes[i % len(lanes)][1]):
                flush.fill_(i & 0xFF)
        lanes[i % len(lanes)][2]()
    t_issue = time.perf_counter() - t0          # host time to issue the K steps (diagnostic)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    del flush
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())

    # ---- per-step latency with batches in flight (p50_ms): the same K steps again, untimed,
    # each bracketed by events on its lane's stream ----
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for i in range(args.steps):
        _, s_i, run_i, _, _ = lanes[i % len(lanes)]
        ev[i][0].record(s_i)
        run_i()
        ev[i][1].record(s_i)
    torch.cuda.synchronize()
    lat_ms = np.array([a.elapsed_time(b) for a, b in ev])

    # ---- per-kernel device time (HIP events on the launch stream), same K steps, one batch
    # at a time (lane 0 alone: kernel averages not inflated by the other lanes' batches) ----
    idx.set_profiling(True)
    for _ in range(args.steps):
        run.prof_run()
    prof = idx.profile()
    idx.set_profiling(False)
    fam_us = {k: 1e3 * v["ms"] / max(args.steps, 1) for k, v in prof.items() if v["launches"]}
    es = 4 if args.dtype == "f32" else 2
    if hybrid:
        r = 50
        flops = 2.0 * B * N_ITEMS * (DIM + r)
        alg_bytes = N_ITEMS * (DIM + r) * es + B * (r * 4 + 8) + B * TOPK * 12 + N_ITEMS // 8
        kname, mpf = scan_kernel_info(args.dtype, DIM, B)
        ab = os.environ.get("BB_AB")
        if args.dtype == "f32" and not (ab and os.environ.get("BB_NO_RR")):
            if ab and os.environ.get("BB_DUAL") == "1":
                kname = ("scan4_dual_kernel<48,8,list|f16> (content d=384 + CF r=50 one-product f16 scans in one "
                         "launch, bounded per-lane candidate lists; exact f32 re-rank of the candidates in the list select)")
            else:
                kname = ("scan4_kernel<48,list|f16> + scan4_kernel<8,list|f16> (content d=384 and CF r=50 one-product "
                         "f16 scans over the packed allowed rows (constraint-first: compact_kernel), one launch per "
                         "side; bounded per-lane candidate lists; exact f32 re-rank of the candidates in the list select)")
    else:
        flops = 2.0 * B * N_ITEMS * DIM
        alg_bytes = N_ITEMS * DIM * es + B * DIM * 4 + B * TOPK * 8    # items + queries + top-K out
        kname, mpf = scan_kernel_info(args.dtype, DIM, B)
    pmc_key = "c3" if hybrid else args.dtype
    step_us = 1e6 * el / args.steps
    mfma16 = args.dtype == "f32" and not (os.environ.get("BB_AB") and os.environ.get("BB_NO_RR"))
    roof = dominant_roofline(fam_us, family_kernels(args.workload, args.dtype, B, kname), flops, alg_bytes, step_us,
                             args.dtype, mpf, pmc_key, mfma16)
    if args.dtype == "f32" and "gemm" in fam_us:
        # (hybrid: both sides, the CF factors padded to 64 f16 columns in the re-rank copy)
        roof["scan_reads"] = scan_read_roofline(B, DIM + (64 if hybrid else 0), fam_us["gemm"])
    if hybrid:
        # constraint-first search: the scans run over the rows the mask allows (packed), so the
        # work they EXECUTE is 2·B·E·(d + r), E = allowed rows; `frac` above prices §8(d)'s
        # full-index work (what the reference's CPU path does per query)
        E = int(np.count_nonzero(q["mask"]))
        ex_flops = 2.0 * B * E * (DIM + 50)
        ex_bytes = E * (DIM + 50) * es + B * (50 * 4 + 8) + B * TOPK * 12
        roof["prefilter"] = {
            "allowed_rows": E, "of_rows": N_ITEMS,
            "executed_flops": ex_flops, "executed_bytes": ex_bytes,
            "executed_frac_of_step_mfma": round(ex_flops / (step_us * 1e-6) / 1e12 / BF16_DENSE_TF, 5),
            "note": "the reference applies the hard constraints first (recommendation_system.py:628-656); "
                    "bb_search packs the allowed rows (compact.hip, one launch) and scans / rescores only them"}

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
    # the same kernels cold: the families' device times with the MALL
    # flushed before every search, so the dominant kernel's frac is an HBM number, not a
    # MALL one (the 39 MB index is Infinity-Cache-resident when warm)
    idx.set_profiling(True)
    n_cold = 20
    for i in range(n_cold):
        with torch.cuda.stream(stream):
            flush.fill_((i + 7) & 0xFF)
        run.prof_run()
        torch.cuda.synchronize()
    prof_c = idx.profile()
    idx.set_profiling(False)
    del flush
    fam_cold = {k: 1e3 * v["ms"] / n_cold for k, v in prof_c.items() if v["launches"] and k in fam_us}
    dom = roof["family"]
    rc_ = roofline(flops, alg_bytes, fam_cold[dom], args.dtype, roof["kernel"], mpf if dom == "gemm" else 1.0, None,
                   mfma16)
    roof["cold"] = {"family": dom, "kernel_us": round(fam_cold[dom], 3), "bound": rc_["bound"],
                    "achieved": rc_["achieved"], "unit": rc_["unit"], "frac": rc_["frac"],
                    "hbm_gbs_at_alg_bytes": rc_["hbm_gbs_at_alg_bytes"],
                    "hbm_frac_at_alg_bytes": rc_["hbm_frac_at_alg_bytes"],
                    "kernels_us_per_step": {k: round(v, 3) for k, v in fam_cold.items()},
                    "note": "the same search with the 256 MiB Infinity Cache flushed (640 MiB fill) before each step; "
                            "warm numbers above are MALL-resident (the index is 39 MB)"}

    if hybrid:
        metric = "similarity queries/sec + p50 latency, hybrid content+CF + mask, 384-d x 25,216 items (configs[2])"
        workload = ("configs[2]: batch=1024 hybrid (liked-set cosine top-100 + CF r=50 top-100, union blend "
                    "0.4/0.6) + constraint mask (num_parts<=800 AND year>=2015) + rated exclusions, top-50")
    else:
        metric = "similarity queries/sec + p50 latency, 384-d x 25,216 items (configs[1])"
        workload = f"configs[1]: batch={B} queries x 25,216 x 384-d items, cosine top-50"
    out = {
        "metric": metric,
        "value": round(world * B * args.steps / el, 1),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * el / args.steps, 4),
        "p50_ms": round(float(np.median(lat_ms)), 4),
        "p50_ms_serial": round(float(np.median(lat_serial)), 4),
        "p50_ms_mall_cold": round(float(np.median(cold)), 4),
        "host_issue_ms_per_step": round(1e3 * t_issue / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (unit-norm N(0,1) rows, seeds 1234 / 4321+rank)",
        "config": {"workload": workload, "items": N_ITEMS, "dim": DIM, "batch": B, "top_k": TOPK,
                   "parallelism": f"replicas x{world}" if world > 1 else "single",
                   "inflight_batches": args.inflight},
        "roofline": roof,
        "kernels_us_per_step": {k: round(v, 3) for k, v in fam_us.items()},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_sweep and not hybrid:
        out["gpu_batch_sweep"] = gpu_batch_sweep(brickrec, base, local, dev)
        out["request_latency"] = request_latency(brickrec, x, dev)
    # rank 0 times the CPU baseline on every line (replicas: the same per-rank workload)
    if rank == 0 and not args.no_cpu and hybrid:
        x_np = x.cpu().numpy()
        cb, ids0 = cpu_baseline_hybrid(x_np, extra["f"], q["mask"], q["liked"], q["rated"], q["u"], TOPK)
        gpu_ids = o_ids.cpu().numpy()
        cb["topk_set_agreement_with_gpu"] = round(float(np.mean([set(gpu_ids[i][gpu_ids[i] >= 0]) == set(ids0[i])
                                                                 for i in range(len(ids0))])), 4)
        out["cpu_baseline"] = cb
    if rank == 0 and not args.no_cpu and not hybrid:
        x_np = x.cpu().numpy()
        q_np = q.cpu().numpy()
        cb, ids0 = cpu_baseline(x_np, q_np, TOPK, budget_s=args.cpu_budget)
        gpu_ids = o_ids.cpu().numpy()
        same = float(np.mean([set(gpu_ids[i]) == set(ids0[i]) for i in range(B)]))
        cb["topk_set_agreement_with_gpu"] = round(same, 4)
        out["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
