"""GPU parity of the bf16 scan with 64 queries per wave (scan4_kernel.h: any bf16 query chunk
taller than 128 rows, padded to whole 256-query groups) against the oracle on the device's
own bf16 operands (exact products, f64 sums): scores within 1e-5, ids exact wherever the
K-th/(K+1)-th gap exceeds f32 accumulation noise.  Covers every query register placement
(d = 768: half of block B in VGPRs; CF r = 50: one k-step), padded query rows, the fused
liked-set gather, per-query exclusions, masks, and the streaming epilogue against the slab
path."""
import numpy as np
import pytest

from oracle import restatement as R

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.fixture(scope="module")
def brickrec():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import brickrec as br
    return br


def _bf16(a):
    """What the device stores for an f32 operand: f64 norm, f32 quotient, RNE -> bf16."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).float().numpy().astype(np.float64)


def _unit_bf16(a):
    a64 = a.astype(np.float64)
    nrm = np.sqrt((a64 * a64).sum(1, keepdims=True))
    nrm[nrm == 0] = 1.0
    return _bf16((a64 / nrm).astype(np.float32))


def _check(sc, ids, sim, k, allowed=None, drop=None):
    """sc/ids against the reference score matrix sim (B x n, f64)."""
    close = 0
    for i in range(sim.shape[0]):
        row = sim[i].copy()
        ok = np.ones(row.shape[0], bool) if allowed is None else allowed(i).copy()
        if drop is not None:
            ok[drop[i]] = False
        ri, rs = R.topk_indices(row, k + 1, ok)
        m = min(k, len(rs))
        np.testing.assert_allclose(sc[i][:m], rs[:m], atol=TOL, rtol=0)
        if len(rs) <= k or rs[k - 1] - rs[k] > 2e-6:
            assert set(ids[i][:m]) == set(ri[:m]), i
        else:
            close += 1
    assert close <= max(2, sim.shape[0] // 20)


def test_scan4_semantic_768_padded_rows(brickrec):
    """d = 768 (configs[3] width, KU = 96: block B half in VGPRs), B = 300 -> two 256-query
    groups with 212 padded rows, slab path."""
    n, d, B, k = 40000, 768, 300, 50
    x = R.unit_rows(n, d, 41)
    q = R.unit_rows(B, d, 42)
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x)
    idx.set_option("stream", 0)
    sc, ids, cnt = idx.search("semantic", k, q_rows=q)
    assert np.all(cnt == k)
    sim = _unit_bf16(q) @ _unit_bf16(x).T
    _check(sc, ids, sim, k)


def test_scan4_similar_gather_mask(brickrec):
    """similar-sets (fused liked-set gather in the scan prologue, rank 0 dropped) with a
    mask, d = 384, B = 512."""
    n, d, B, k = 30000, 384, 512, 40
    x = R.unit_rows(n, d, 43)
    rng = np.random.default_rng(44)
    qi = rng.choice(n, B, replace=False)
    mask = rng.random(n) < 0.5
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x)
    idx.set_option("stream", 0)
    sc, ids, cnt = idx.search("similar", k, q_items=qi, mask=mask)
    xs = _unit_bf16(x)
    sim = xs[qi] @ xs.T
    # rank 0 = the unmasked arg-max (the item itself: no duplicate rows here)
    _check(sc, ids, sim, k, allowed=lambda i: mask, drop=qi)
    for i in range(B):
        assert qi[i] not in set(ids[i])


def test_scan4_cf_excl_mask(brickrec):
    """CF (r = 50 -> one 16-wide k step per block) with per-query exclusions and a mask."""
    n, r, B, k = 20000, 50, 256, 30
    rng = np.random.default_rng(45)
    x = R.unit_rows(n, 64, 46)
    f = rng.normal(0, 0.1, (n, r)).astype(np.float32)
    u = rng.normal(0, 0.1, (B, r)).astype(np.float32)
    mask = rng.random(n) < 0.6
    excl = rng.random((B, n)) < 0.02
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x)
    idx.upload_cf(f)
    idx.set_option("stream", 0)
    sc, ids, cnt = idx.search("cf", k, q_cf=u, mask=mask, excl=excl)
    sim = _bf16(u) @ _bf16(f).T
    _check(sc, ids, sim, k, allowed=lambda i: mask & ~excl[i])
    for i in range(B):
        assert not excl[i][ids[i][:cnt[i]]].any()


def test_scan4_stream_equals_slab(brickrec):
    """Streaming epilogue (two streams of candidates per lane) == slab path, and both
    against the reference: bf16 384-d, B = 768 (three groups), similar-sets with a mask."""
    n, d, B, k = 150000, 384, 768, 100
    x = R.unit_rows(n, d, 47)
    rng = np.random.default_rng(48)
    qi = rng.choice(n, B, replace=False)
    mask = rng.random(n) < 0.7
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x)
    idx.set_option("stream", 1)
    idx.set_profiling(True)
    a = idx.search("similar", k, q_items=qi, mask=mask)
    prof = idx.profile()
    idx.set_profiling(False)
    assert prof["rerun"]["launches"] == 0, prof  # finished on the streaming path
    assert prof["gemm"]["launches"] >= 2, prof   # pilot + streaming pass(es)
    idx.set_option("stream", 0)
    b = idx.search("similar", k, q_items=qi, mask=mask)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)
    xs = _unit_bf16(x)
    sel = np.arange(0, B, 37)
    sim = xs[qi[sel]] @ xs.T
    _check(a[0][sel], a[1][sel], sim, k, allowed=lambda i: mask, drop=qi[sel])


def test_scan4_hybrid_bf16_stream_and_slab(brickrec):
    """bf16 hybrid (content similar-sets + CF with rated exclusions, under a mask), B = 300
    -> both sides on scan4; streaming forced == slab, and both against the union blend of
    the reference restatement over the device's bf16 operands (finalize1 path)."""
    n, d, r, B, k = 120000, 384, 50, 300, 20
    x = R.unit_rows(n, d, 71)
    rng = np.random.default_rng(72)
    f = rng.normal(0, 0.1, (n, r)).astype(np.float32)
    u = rng.normal(0, 0.1, (B, r)).astype(np.float32)
    mask = rng.random(n) < 0.5
    rated = rng.random((B, n)) < 0.01
    qi = rng.choice(n, B, replace=False)
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x)
    idx.upload_cf(f)
    kw = dict(q_items=qi, q_cf=u, mask=mask, excl=rated)
    idx.set_option("stream", 1)
    idx.set_profiling(True)
    a = idx.search("hybrid", k, **kw)
    prof = idx.profile()
    idx.set_profiling(False)
    assert prof["rerun"]["launches"] == 0, prof
    idx.set_option("stream", 0)
    b = idx.search("hybrid", k, **kw)
    for p_, q_ in zip(a, b):
        assert np.array_equal(p_, q_)
    xs, fs, us = _unit_bf16(x), _bf16(f), _bf16(u)
    close = 0
    for i in range(0, B, 23):
        cs = xs[qi[i]] @ xs.T
        ok = mask.copy()
        ok[int(np.argmax(cs))] = False          # rank 0: the unmasked arg-max
        c_i, c_s = R.topk_indices(cs, 2 * k, ok)
        f_i, f_s = R.topk_indices(fs @ us[i], 2 * k, mask & ~rated[i])
        ri, rsc = R.union_blend(c_i, c_s, f_i, f_s, 0.4, 0.6, k + 1)
        np.testing.assert_allclose(a[0][i], rsc[:k], atol=TOL, rtol=0)
        if len(rsc) <= k or rsc[k - 1] - rsc[k] > 2e-6:
            assert set(a[1][i]) == set(ri[:k]), i
        else:
            close += 1
    assert close <= 2
