"""GPU parity of the streaming top-K path (large indexes: pilot bound + candidate regions,
no B×n score slab) against the oracle and against the slab path on the same index.

Both paths run the same scan kernels, so their scores are bitwise equal and the lists must
match exactly; against the numpy oracle the bar is the north_star one (ids exact where the
K-th/(K+1)-th gap exceeds fp32 summation noise, scores within 1e-5).
"""
import numpy as np
import pytest

from oracle import restatement as R
from _parity import GAP, Gate, check_row

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.fixture(scope="module")
def brickrec():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import brickrec as br
    return br


def _both(idx, mode, k, stream_gemms=None, **kw):
    """(stream results, slab results) of one search.  The streaming search must finish on
    the streaming path: no overflow handed back to the slab path (profile "rerun"), and at
    least stream_gemms scan launches (pilot + streaming passes per side and query chunk;
    the two-level bound adds a pass on indexes >= 4x the pilot)."""
    idx.set_option("stream", 1)
    idx.set_profiling(True)
    a = idx.search(mode, k, **kw)
    prof = idx.profile()
    idx.set_profiling(False)
    assert prof["rerun"]["launches"] == 0, prof
    if stream_gemms is not None:
        assert prof["gemm"]["launches"] >= stream_gemms, prof
    idx.set_option("stream", 0)
    b = idx.search(mode, k, **kw)
    idx.set_option("stream", -1)
    return a, b


def _same(a, b, exact=True):
    """Stream vs slab results.  A bf16 index runs the same scan kernels on both paths, so the
    lists are bitwise equal.  An f32 index streams through the split-precision scan (fp32-
    class, |error| ~1e-7) while its one-slab search runs the exact re-rank, so there the
    scores agree within 1e-6 and the ids wherever adjacent scores are further apart."""
    if exact:
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
        return
    (sa, ia, ca), (sb, ib, cb) = a, b
    assert np.array_equal(ca, cb)
    np.testing.assert_allclose(sa, sb, atol=1e-6, rtol=0)
    for i in range(len(ca)):
        c = int(ca[i])
        if c > 1 and np.all(-np.diff(sb[i][:c].astype(np.float64)) > 2e-6):
            assert list(ia[i][:c]) == list(ib[i][:c]), i
        elif c:
            sure = set(ib[i][:c][sb[i][:c] > sb[i][c - 1] + 2e-6])
            assert sure <= set(ia[i][:c]), i


def test_stream_semantic_f32_vs_oracle(brickrec):
    n, d, B, k = 150000, 384, 300, 100
    x = R.unit_rows(n, d, 1234)
    q = R.unit_rows(B, d, 4321)
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    (sc, ids, cnt), slab = _both(idx, "semantic", k, stream_gemms=2, q_rows=q)
    _same((sc, ids, cnt), slab, exact=False)
    assert np.all(cnt == k)
    sim = R.cosine_scores(q, x).astype(np.float64)
    gate = Gate("stream f32 150K x 384 semantic top-100")
    for i in range(B):
        ri, rs = R.topk_indices(sim[i], k + 1)
        check_row(gate, sc[i], ids[i], ri[:k], rs[:k], k, rs[k])
    gate.report(0.1)


def test_stream_similar_bf16_mask(brickrec):
    """bf16 768-d (configs[3] width), similar-sets with a mask: rank 0 (the query item)
    is dropped, masked items never appear; stream == slab exactly."""
    n, d, B, k = 120000, 768, 130, 50
    x = R.unit_rows(n, d, 5)
    rng = np.random.default_rng(9)
    mask = rng.random(n) < 0.3
    qi = rng.choice(n, B, replace=False)
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x)
    (sc, ids, cnt), slab = _both(idx, "similar", k, stream_gemms=2, q_items=qi, mask=mask)
    _same((sc, ids, cnt), slab)
    assert np.all(cnt == k)
    for i in range(B):
        assert qi[i] not in set(ids[i])
        assert mask[ids[i]].all()
        assert np.all(np.diff(sc[i]) <= 0)
    # oracle over the stored bf16 rows (exact products, f64 sums): rank 0 of the unmasked row
    # dropped, then the masked top-k (recommendation_system.py:217, 229)
    rows = idx.get_rows(np.arange(n)).astype(np.float64)
    sim = rows[qi[::4]] @ rows.T
    gate = Gate("stream bf16 120K x 768 similar + mask")
    for j, i in enumerate(range(0, B, 4)):
        ok = mask.copy()
        ok[R.rank0(sim[j])] = False
        ri, rs = R.topk_indices(sim[j], k + 1, ok)
        check_row(gate, sc[i], ids[i], ri[:k], rs[:k], k, rs[k])
    gate.report(0.1)


def test_stream_hybrid_cf_excl(brickrec):
    """hybrid: content (drop rank 0) + CF (rated excluded) sides, both streamed."""
    n, d, r, B, k = 110000, 128, 50, 64, 20
    x = R.unit_rows(n, d, 17)
    rng = np.random.default_rng(4)
    f = rng.normal(0, 0.1, (n, r))
    u = rng.normal(0, 0.1, (B, r))
    mask = rng.random(n) < 0.4
    excl = rng.random((B, n)) < 0.01
    qi = rng.choice(n, B, replace=False)
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    idx.upload_cf(f)
    a, b = _both(idx, "hybrid", k, stream_gemms=4, q_items=qi, q_cf=u, mask=mask, excl=excl)
    _same(a, b, exact=False)
    hyb = a
    a, b = _both(idx, "cf", k, stream_gemms=2, q_cf=u, mask=mask, excl=excl)
    _same(a, b, exact=False)
    sc, ids, cnt = a
    for i in range(0, B, 7):
        ri, rs = R.cf_topk(u[i], f, k, mask & ~excl[i])
        np.testing.assert_allclose(sc[i][:len(rs)], rs, atol=TOL, rtol=0)
    # hybrid leg vs the oracle: content top-2k (rank 0 dropped, mask) and CF top-2k (rated
    # skipped, mask), union blend 0.4 / 0.6 (recommendation_system.py:646-668, 789-843)
    hs_, hi_, hc_ = hyb
    xn = R.normalize_rows(x)
    gate = Gate("stream hybrid 110K f32 + mask + excl")
    for i in range(0, B, 3):
        s_c = (xn[qi[i]] @ xn.T).astype(np.float64)
        okc = mask.copy()
        okc[R.rank0(s_c)] = False
        ci, cs = R.topk_indices(s_c, 2 * k + 1, okc)
        fi, fs = R.topk_indices(f @ u[i], 2 * k + 1, mask & ~excl[i])
        bi, bs = R.union_blend(ci[:2 * k], cs[:2 * k], fi[:2 * k], fs[:2 * k], 0.4, 0.6, k + 1)
        if cs[2 * k - 1] - cs[2 * k] <= GAP or fs[2 * k - 1] - fs[2 * k] <= GAP:
            gate.gated += 1
            continue
        check_row(gate, hs_[i], hi_[i], bi[:k], bs[:k], k, bs[k])
    gate.report(0.1)


def test_stream_two_query_chunks(brickrec):
    """B > 1024: two query chunks of different padded heights (different region layouts)."""
    n, d, B, k = 100000, 64, 1100, 30
    x = R.unit_rows(n, d, 23)
    q = R.unit_rows(B, d, 24)
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    # a 16 MiB workspace cannot hold 1100 pilot rows: query chunks of 512, 512 and 76 (ragged)
    idx.set_option("workspace_bytes", 16 << 20)
    (sc, ids, cnt), slab = _both(idx, "semantic", k, stream_gemms=6, q_rows=q)
    _same((sc, ids, cnt), slab, exact=False)
    sim = R.cosine_scores(q[-5:], x).astype(np.float64)
    for j in range(5):
        ri, rs = R.topk_indices(sim[j], k)
        np.testing.assert_allclose(sc[B - 5 + j], rs, atol=TOL, rtol=0)


def test_stream_overflow_falls_back(brickrec):
    """All-equal scores (a zero query): every item reaches the bound, the candidate regions
    overflow and the search reruns on the slab path — ids ascending, scores 0."""
    n, d, k = 100000, 64, 10
    x = R.unit_rows(n, d, 29)
    q = np.concatenate([np.zeros((1, d), np.float32), R.unit_rows(3, d, 30)])
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    idx.set_option("stream", 1)
    sc, ids, cnt = idx.search("semantic", k, q_rows=q)
    assert list(ids[0]) == list(range(k)) and np.all(sc[0] == 0)
    sim = R.cosine_scores(q[1:], x).astype(np.float64)
    for j in range(3):
        ri, rs = R.topk_indices(sim[j], k)
        np.testing.assert_allclose(sc[1 + j], rs, atol=TOL, rtol=0)


def test_stream_small_index_forced(brickrec):
    """Forced streaming on an index smaller than the pilot minimum (pilot = whole index)."""
    n, d, B, k = 3000, 384, 40, 25
    x = R.unit_rows(n, d, 31)
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    qi = np.arange(B) * 7
    a, b = _both(idx, "similar", k, stream_gemms=2, q_items=qi)
    _same(a, b, exact=False)
    for i in range(0, B, 9):
        ri, rs = R.similar_sets(x, int(qi[i]), k)
        assert list(a[1][i]) == list(ri)


def test_stream_large_bf16_torch_upload(brickrec):
    """configs[4]-shaped shard (bf16, 384-d, top-100, similar-sets) uploaded straight from a torch tensor
    into device memory a previous index just released: the upload must see the finished
    rows (the library converts on its own stream), so the pilot bound is real and the
    streaming pass finishes without a region overflow; stream == slab exactly, and the
    scores match an f64 reference over the stored bf16 rows."""
    import torch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(77)
    old = brickrec.ItemIndex(dtype="bf16")
    y = torch.randn((50000, 384), generator=g, device=dev)
    old.upload_items(y)
    old.search("semantic", 10, q_rows=y[:8])
    old.close()
    del y, old
    torch.cuda.empty_cache()
    n, d, B, k = 400000, 384, 256, 100
    x = torch.randn((n, d), generator=g, device=dev)
    x = x / x.norm(dim=1, keepdim=True)
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x, prenormalized=True)     # no explicit sync by the caller
    qi = torch.randperm(n, generator=g, device=dev)[:B]
    (sc, ids, cnt), slab = _both(idx, "similar", k, stream_gemms=2, q_items=qi)
    torch.cuda.synchronize()
    for u, v in zip((sc, ids, cnt), slab):
        assert torch.equal(u, v)
    # reference over the stored bf16 rows (exact products, f64 sums); rank 0 = the item itself
    rows = idx.get_rows(torch.arange(n, device=dev)).double()
    ref = rows[qi[:32]] @ rows.T
    ref[torch.arange(32, device=dev), qi[:32]] = -float("inf")
    rs, ri = torch.topk(ref, k + 1, dim=1)
    assert torch.max(torch.abs(sc[:32].double() - rs[:, :k])).item() < 1e-5
    for i in range(32):
        if (rs[i, k - 1] - rs[i, k]).item() > 1e-5:
            assert set(ids[i].tolist()) == set(ri[i, :k].tolist())


@pytest.mark.parametrize("dtype,mode", [("bf16", "similar"), ("f32", "semantic")])
def test_stream_two_level_bound(brickrec, dtype, mode):
    """Two-level streaming bound: a workspace too small for a 1/16 pilot leaves the pilot
    at 8192 rows of 200,000 (n >= 16·n0), so the stream runs pass A over [0, n1), an exact
    candidate select of that range whose last key bounds pass B over [n1, n), and a final
    select over pass B's candidates plus pass A's list (rank 0 carried across).  Three scan
    launches, no slab rerun, and the lists equal the slab path's exactly."""
    n, d, B, k = 200000, 384, 256, 50
    x = R.unit_rows(n, d, 61)
    rng = np.random.default_rng(62)
    mask = rng.random(n) < 0.6
    idx = brickrec.ItemIndex(dtype=dtype)
    idx.upload_items(x)
    idx.set_option("workspace_bytes", 8 << 20)
    idx.set_option("stream_refine", 1)   # auto takes it from 500K rows
    if mode == "similar":
        qi = rng.choice(n, B, replace=False)
        kw = dict(q_items=qi, mask=mask)
    else:
        kw = dict(q_rows=R.unit_rows(B, d, 63), mask=mask)
    idx.set_option("stream", 1)
    idx.set_profiling(True)
    a = idx.search(mode, k, **kw)
    prof = idx.profile()
    idx.set_profiling(False)
    assert prof["rerun"]["launches"] == 0, prof
    assert prof["gemm"]["launches"] == 3, prof
    assert prof["select"]["launches"] == 3, prof   # pilot slab, pass A list, final
    idx.set_option("stream", 0)
    b = idx.search(mode, k, **kw)
    _same(a, b, exact=dtype == "bf16")
    assert np.all(a[2] == k)
    if mode == "similar":
        for i in range(B):
            assert qi[i] not in set(a[1][i]) and mask[a[1][i]].all()


def test_stream_ties_at_kth(brickrec):
    """Every row present 24 times (bf16, 384-d; the copies spread over the index, so no
    candidate region collects them all): equal scores straddle the K-th place of almost
    every query, so the candidate select's second bisection (item word among equal score
    images) decides the list; stream == slab exactly (ids ascending among equals)."""
    base = R.unit_rows(5000, 384, 71)
    x = np.tile(base, (24, 1))                 # 120,000 rows
    q = R.unit_rows(160, 384, 72)
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x)
    (sc, ids, cnt), slab = _both(idx, "semantic", 50, stream_gemms=2, q_rows=q)
    _same((sc, ids, cnt), slab)
    assert np.all(cnt == 50)
    ties = sum(int(np.sum(sc[i] == sc[i][-1])) > 1 for i in range(len(q)))
    assert ties > len(q) // 2, ties   # the tie path ran for most rows


def test_stream_many_candidates_paged(brickrec):
    """top-300 (K_int 301): ~8·K_int = 2,400 candidates per query, more than the 2,048 a
    wave of the candidate select holds in registers — the paged bisection; stream == slab
    exactly on a bf16 index (the slab path selects from the score image, not from candidates)."""
    n, d, B, k = 125000, 768, 96, 300
    x = R.unit_rows(n, d, 73)
    q = R.unit_rows(B, d, 74)
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x)
    (sc, ids, cnt), slab = _both(idx, "semantic", k, stream_gemms=2, q_rows=q)
    _same((sc, ids, cnt), slab)
    assert np.all(cnt == k)
    for i in range(0, B, 16):
        assert np.all(np.diff(sc[i]) <= 0)
        assert set(ids[i]) == set(np.unique(ids[i]))


def test_stream_small_pilot_pages(brickrec):
    """A 2 MiB workspace holds a pilot of a few thousand rows of 125,000: ~30·K_int = 3,000
    candidates per query for top-100 — two 2,048-key pages of the candidate select, each
    reduced to its top K_int before the final bisection; stream == slab exactly (bf16)."""
    n, d, B, k = 125000, 768, 96, 100
    x = R.unit_rows(n, d, 75)
    q = R.unit_rows(B, d, 76)
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x)
    idx.set_option("workspace_bytes", 2 << 20)
    (sc, ids, cnt), slab = _both(idx, "semantic", k, stream_gemms=2, q_rows=q)
    _same((sc, ids, cnt), slab)
    assert np.all(cnt == k)


def test_stream_refine_short_carry_paged(brickrec):
    """Two-level bound where a selective mask leaves pass A's list (the carry) with fewer than
    K real keys, and pass B more than 2,048 candidates: the final candidate select pages
    (1,024 keys) and its last page holds more than K keys but fewer than K real ones (the
    carry's empty keys at its end).  Each page must return at most K keys (the
    page's K-th key was 0 there and every slot was taken, past the wave's LDS list)."""
    n, d, B, k = 200000, 384, 64, 50
    x = R.unit_rows(n, d, 81)
    q = R.unit_rows(B, d, 82)
    mask = np.zeros(n, bool)
    mask[np.arange(10) * 97] = True                                  # pass A: 10 eligible
    mask[np.linspace(100000, n - 1, 2068).astype(np.int64)] = True   # pass B: 2,068
    idx = brickrec.ItemIndex(dtype="bf16")
    idx.upload_items(x)
    idx.set_option("workspace_bytes", 2 << 20)   # pilot 8,192 rows: n1 ~ 40K < 100K
    idx.set_option("stream_refine", 1)
    idx.set_option("stream", 1)
    idx.set_profiling(True)
    a = idx.search("semantic", k, q_rows=q, mask=mask)
    prof = idx.profile()
    idx.set_profiling(False)
    assert prof["rerun"]["launches"] == 0, prof
    assert prof["gemm"]["launches"] == 3, prof
    idx.set_option("stream", 0)
    b = idx.search("semantic", k, q_rows=q, mask=mask)
    _same(a, b)
    sc, ids, cnt = a
    assert np.all(cnt == k)
    rows = idx.get_rows(np.arange(n)).astype(np.float64)
    sim = R.normalize_rows(q).astype(np.float64) @ rows.T
    for i in range(0, B, 8):
        assert mask[ids[i]].all() and len(set(ids[i])) == k
        ri, rs = R.topk_indices(sim[i], k, mask)
        # bf16 query operand vs the f32 query here: ~1e-3 apart
        np.testing.assert_allclose(sc[i], rs, atol=5e-3, rtol=0)
