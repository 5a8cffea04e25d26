"""GPU parity at the shapes of every BASELINE.json config, through the C-ABI.

* configs[0]: B=1, top-10, 25,216 x 384 f32 — semantic and similar against the oracle.
* configs[2]: hybrid, f32, 25,216 x 384 content + r=50 CF, B=1024, top-50, the §8(d)
  constraint mask (num_parts <= 800 AND year >= 2015, evaluated on the device) and
  per-user rated exclusions — every query against the oracle's union blend of its content
  and CF top-2k lists (recommendation_system.py:612-677, 789-843).
* configs[3]: 1M x 768 bf16, B=4096, top-100 — unsharded vs 8 row shards on one device
  (search_keys + finalize, the RCCL merge's device half), bit-identical; scores and ids
  against an f64 recompute over the stored rows for 64 queries.
* configs[4]: 10M x 384 bf16, B=8192, top-100 — the same checks, the f64 recompute
  chunked on the device.
* A sharded f32 hybrid (mask + exclusions) whose shards take the streaming path, against
  the unsharded search bit for bit and against the oracle.

Near-tie gating (tests/_parity.py) is reported per test and bounded.
"""
import numpy as np
import pytest

from oracle import restatement as R
from _parity import GAP, TOL, Gate, blend_sure, check_row

pytestmark = pytest.mark.gpu
N25, D25 = 25216, 384


@pytest.fixture(scope="module")
def brickrec():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import brickrec as br
    return br


@pytest.fixture(scope="module")
def items25():
    x = R.unit_rows(N25, D25, 1234)
    return x, R.normalize_rows(x)


# --------------------------------------------------------------------------- configs[0]
def test_c0_single_query_top10(brickrec, items25):
    x, xn = items25
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    gate = Gate("configs[0] semantic+similar B=1 top-10")
    for seed in range(8):
        q = R.unit_rows(1, D25, 4321 + seed)
        sc, ids, cnt = idx.search("semantic", 10, q_rows=q)
        sim = R.cosine_scores(q, x)[0].astype(np.float64)
        ri, rs = R.topk_indices(sim, 11)
        check_row(gate, sc[0], ids[0], ri[:10], rs[:10], 10, rs[10])
        item = seed * 3001
        sc, ids, cnt = idx.search("similar", 10, q_items=[item])
        sim = (xn[item:item + 1] @ xn.T)[0].astype(np.float64)
        ok = np.ones(N25, bool)
        ok[R.rank0(sim)] = False
        ri, rs = R.topk_indices(sim, 11, ok)
        check_row(gate, sc[0], ids[0], ri[:10], rs[:10], 10, rs[10])
    gate.report(0.25)


# --------------------------------------------------------------------------- configs[2]
def _c2_data():
    rng = np.random.default_rng(2024)
    r, B = 50, 1024
    f = rng.normal(0.0, 0.1, (N25, r))
    u = rng.normal(0.0, 0.1, (B, r))
    parts = rng.integers(1, 6000, N25).astype(np.int32)
    year = rng.integers(1949, 2025, N25).astype(np.int16)
    theme = rng.integers(0, 400, N25).astype(np.int32)
    liked = rng.choice(N25, B, replace=False)
    rated = np.zeros((B, N25), bool)
    for b in range(B):
        rated[b, rng.choice(N25, int(rng.integers(10, 31)), replace=False)] = True
    return f, u, parts, year, theme, liked, rated


def test_c2_hybrid_mask_b1024(brickrec, items25):
    """configs[2] at its own shape: device mask, device HYBRID (two sides, union blend)."""
    x, xn = items25
    f, u, parts, year, theme, liked, rated = _c2_data()
    B, k, ks = len(liked), 50, 100
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    idx.upload_cf(f)
    idx.upload_attrs(parts, year, theme)
    mask = idx.eval_mask(brickrec.Predicate(parts_max=800, year_min=2015))
    assert np.array_equal(mask, (parts <= 800) & (year >= 2015) & (parts > 0))
    sc, ids, cnt = idx.search("hybrid", k, q_items=liked, q_cf=u, mask=mask, excl=rated)

    # oracle: content top-2k of each liked set (rank 0 of the unmasked row dropped, then the
    # mask walk), CF top-2k (rated skipped, mask), union blend 0.4 / 0.6 in f64
    sim_c = (xn[liked] @ xn.T).astype(np.float64)
    sim_f = u @ f.T
    gate = Gate("configs[2] hybrid B=1024 + mask")
    n_sure = 0
    for b in range(B):
        okc = mask.copy()
        okc[R.rank0(sim_c[b])] = False
        ci, cs = R.topk_indices(sim_c[b], ks + 8, okc)
        okf = mask & ~rated[b]
        fi, fs = R.topk_indices(sim_f[b], ks + 8, okf)
        hi, hs = R.union_blend(ci[:ks], cs[:ks], fi[:ks], fs[:ks], 0.4, 0.6, k + 1)
        # the union's membership depends on both side boundaries: gate on all three
        side_tie = (len(ci) > ks and cs[ks - 1] - cs[ks] <= GAP) or (len(fi) > ks and fs[ks - 1] - fs[ks] <= GAP)
        L = min(k, len(hi))
        if side_tie:
            # a near-tied side boundary leaves some union memberships open: every blended item
            # whose membership does not depend on it must still be in the list, with its score
            gate.gated += 1
            assert np.all(np.diff(sc[b][:cnt[b]]) <= 0)
            sure = blend_sure(ci, cs, fi, fs, ks, 0.4, 0.6, k)
            got = {int(i): float(s) for i, s in zip(ids[b][:cnt[b]], sc[b][:cnt[b]])}
            assert set(sure) <= set(got), (b, sorted(set(sure) - set(got)))
            for i, h in sure.items():
                assert abs(got[i] - h) <= TOL, (b, i, got[i], h)
            n_sure += len(sure)
            continue
        check_row(gate, sc[b], ids[b], hi[:L], hs[:L], k, hs[k] if len(hi) > k else None)
        assert cnt[b] == L
    print(f"[parity] configs[2] gated queries: {n_sure} blended items checked for membership")
    gate.report(0.05)


# --------------------------------------------------------------------------- configs[3] / [4]
def _unit_rows_dev(n, d, seed, dev, chunk=1 << 20):
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    out = torch.empty((n, d), dtype=torch.float32, device=dev)
    for i in range(0, n, chunk):
        t = torch.randn((min(chunk, n - i), d), generator=g, device=dev)
        out[i:i + t.shape[0]] = t / t.norm(dim=1, keepdim=True)
    return out


def _bf16_query_operand(q):
    """The device's semantic query operand for a bf16 index: f64 norm, f32 quotient, RNE bf16."""
    q64 = q.double()
    return (q64 / q64.norm(dim=1, keepdim=True)).float().bfloat16().double()


def _f64_topk(idx, qop, n, k, chunk):
    """Exact top-(k+1) of qop · rows^T over the index's stored rows, in f64, chunked."""
    import torch
    dev = qop.device
    best_s = best_i = None
    for c0 in range(0, n, chunk):
        ids = torch.arange(c0, min(n, c0 + chunk), device=dev)
        s = qop @ idx.get_rows(ids).double().T
        ts, ti = torch.topk(s, min(k + 1, s.shape[1]), dim=1)
        ti = ti + c0
        if best_s is None:
            best_s, best_i = ts, ti
        else:
            cs, ci = torch.cat([best_s, ts], 1), torch.cat([best_i, ti], 1)
            best_s, j = torch.topk(cs, k + 1, dim=1)
            best_i = torch.gather(ci, 1, j)
    return best_s.cpu().numpy(), best_i.cpu().numpy()


def _sharded_vs_unsharded(brickrec, x, q, k, P, n_check, chunk, name):
    import torch
    dev = x.device
    n, d = x.shape
    B = q.shape[0]
    full = brickrec.ItemIndex(dtype="bf16")
    full.upload_items(x)
    full.set_profiling(True)
    sc, ids, cnt = full.search("semantic", k, q_rows=q)
    torch.cuda.synchronize()
    prof = full.profile()
    full.set_profiling(False)
    assert prof["rerun"]["launches"] == 0, prof        # finished on the streaming path
    assert bool((cnt == k).all())
    assert bool((sc[:, 1:] <= sc[:, :-1]).all())       # descending lists
    # every stored row against torch's own conversion (f64 norm, f32 quotient, RNE bf16), so
    # the f64 recompute below, which reads the stored rows, is anchored outside the library.
    # The two f64 norms may sum in different orders: a differing element would have to sit
    # within 2^-52 of a bf16 rounding boundary (~n·d·2^-44 of them expected), so any
    # difference must be a single bf16 ulp and there may be at most a handful.
    n_diff = 0
    for c0 in range(0, n, chunk):
        ids_c = torch.arange(c0, min(n, c0 + chunk), device=dev)
        got = full.get_rows(ids_c).view(torch.int16).int()
        want = _bf16_query_operand(x[c0:c0 + chunk]).bfloat16().view(torch.int16).int()
        dif = (got - want).abs()
        assert int(dif.max()) <= 1, (name, c0, int(dif.max()))
        n_diff += int((dif != 0).sum())
    assert n_diff <= 8, (name, n_diff)
    print(f"[parity] {name}: {n} stored bf16 rows vs torch conversion, {n_diff} elements differ by 1 ulp")
    # f64 recompute for n_check queries spread over the batch (every query: round 5), on the
    # device in 64K-row chunks (B x 65,536 f64 scores at a time)
    rows_q = torch.linspace(0, B - 1, n_check, device=dev).long()
    rs, ri = _f64_topk(full, _bf16_query_operand(q[rows_q]), n, k, 1 << 16)
    sc_h, ids_h = sc[rows_q].cpu().numpy(), ids[rows_q].cpu().numpy()
    gate = Gate(name)
    for j in range(n_check):
        check_row(gate, sc_h[j], ids_h[j], ri[j, :k], rs[j, :k], k, rs[j, k], order=False)
    gate.report(0.1)
    full.close()
    del full
    torch.cuda.empty_cache()
    # the same batch over P row shards on one device, merged by bb_finalize
    per = (n + P - 1) // P
    keys, maxk, last = [], [], None
    for p in range(P):
        lo, hi = p * per, min(n, (p + 1) * per)
        sh = brickrec.ItemIndex(dtype="bf16", id_offset=lo)
        sh.upload_items(x[lo:hi])
        kk, mk = sh.search_keys("semantic", k, q_rows=q)
        keys.append(kk)
        maxk.append(mk)
        torch.cuda.synchronize()
        if last is not None:
            last.close()
        last = sh
    ssc, sids, scnt = last.finalize("semantic", k, torch.stack(keys), torch.stack(maxk), P)
    torch.cuda.synchronize()
    assert torch.equal(sids, ids), "sharded ids differ from the unsharded search"
    assert torch.equal(ssc, sc), "sharded scores differ from the unsharded search"
    assert torch.equal(scnt, cnt)
    last.close()


def test_c3_1M_768_bf16_b4096_sharded(brickrec):
    import torch
    dev = torch.device("cuda", 0)
    x = _unit_rows_dev(1_000_000, 768, 1234, dev)
    q = _unit_rows_dev(4096, 768, 4321, dev)
    _sharded_vs_unsharded(brickrec, x, q, 100, 8, 4096, 1 << 18, "configs[3] 1M x 768 bf16 B=4096 top-100")


def test_c4_10M_384_bf16_b8192_sharded(brickrec):
    import torch
    dev = torch.device("cuda", 0)
    x = _unit_rows_dev(10_000_000, 384, 1234, dev)
    q = _unit_rows_dev(8192, 384, 4321, dev)
    _sharded_vs_unsharded(brickrec, x, q, 100, 8, 8192, 1 << 20, "configs[4] 10M x 384 bf16 B=8192 top-100")


# --------------------------------------------------------------------------- sharded hybrid
def test_sharded_hybrid_streaming_vs_unsharded_and_oracle(brickrec):
    """f32 hybrid with mask + exclusions over 2 row shards of 125K rows (streaming path on
    each shard): bb_finalize's merge == the unsharded search bit for bit, and both match the
    oracle's union blend."""
    import torch
    from brickrec.engine import bits_from_bool
    dev = torch.device("cuda", 0)
    n, d, r, B, k = 250_000, 128, 50, 48, 20
    x = R.unit_rows(n, d, 41)
    rng = np.random.default_rng(42)
    f = rng.normal(0, 0.1, (n, r)).astype(np.float32)
    u = rng.normal(0, 0.1, (B, r)).astype(np.float32)
    mask = rng.random(n) < 0.5
    excl = rng.random((B, n)) < 0.002
    liked = rng.choice(n, B, replace=False)
    full = brickrec.ItemIndex(dtype="f32")
    full.upload_items(x)
    full.upload_cf(f)
    sc, ids, cnt = full.search("hybrid", k, q_items=liked, q_cf=u, mask=mask, excl=excl)
    qrows = torch.from_numpy(full.get_rows(liked)).to(dev)   # feat_matrix[target] of each liked set
    cut = n // 2
    keys, maxk = [], []
    for lo, hi in ((0, cut), (cut, n)):
        sh = brickrec.ItemIndex(dtype="f32", id_offset=lo)
        sh.upload_items(x[lo:hi])
        sh.upload_cf(f[lo:hi])
        sh.set_profiling(True)
        mw = torch.from_numpy(bits_from_bool(mask[lo:hi]).view(np.int32)).to(dev)
        ew = torch.from_numpy(bits_from_bool(excl[:, lo:hi]).view(np.int32)).to(dev)
        kk, mk = sh.search_keys("hybrid", k, q_rows=qrows, q_cf=torch.from_numpy(u).to(dev), mask=mw, excl=ew)
        torch.cuda.synchronize()
        prof = sh.profile()
        assert prof["gemm"]["launches"] >= 4 and prof["rerun"]["launches"] == 0, prof   # streamed, both sides
        keys.append(kk)
        maxk.append(mk)
    ssc, sids, scnt = sh.finalize("hybrid", k, torch.stack(keys), torch.stack(maxk), 2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(sids.cpu().numpy(), ids)
    np.testing.assert_array_equal(ssc.cpu().numpy(), sc)
    np.testing.assert_array_equal(scnt.cpu().numpy(), cnt)
    xn = R.normalize_rows(x)
    gate = Gate("sharded hybrid 250K f32 + mask + excl")
    for b in range(B):
        sim = (xn[liked[b]] @ xn.T).astype(np.float64)
        okc = mask.copy()
        okc[R.rank0(sim)] = False
        ci, cs = R.topk_indices(sim, 2 * k + 1, okc)
        fsc = f.astype(np.float64) @ u[b].astype(np.float64)
        fi, fs = R.topk_indices(fsc, 2 * k + 1, mask & ~excl[b])
        hi_, hs = R.union_blend(ci[:2 * k], cs[:2 * k], fi[:2 * k], fs[:2 * k], 0.4, 0.6, k + 1)
        if cs[2 * k - 1] - cs[2 * k] <= GAP or fs[2 * k - 1] - fs[2 * k] <= GAP:
            gate.gated += 1
            assert np.all(np.diff(sc[b]) <= 0)
            ci, cs = R.topk_indices(sim, 2 * k + 8, okc)
            fi, fs = R.topk_indices(fsc, 2 * k + 8, mask & ~excl[b])
            got = {int(i): float(s) for i, s in zip(ids[b], sc[b]) if i >= 0}
            for i, h in blend_sure(ci, cs, fi, fs, 2 * k, 0.4, 0.6, k).items():
                assert i in got and abs(got[i] - h) <= TOL, (b, i)
            continue
        check_row(gate, sc[b], ids[b], hi_[:k], hs[:k], k, hs[k])
    gate.report(0.1)
