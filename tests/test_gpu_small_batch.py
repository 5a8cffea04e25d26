"""GPU parity of the small-batch exact search (csrc/sq.hip): batches of <= 16 query rows of one
side on an f32 index take ONE pass over the f32 rows with every score exact (f32 products
summed in f64 in rescore_rows' fixed order, rounded to f32) — the reference's own request
shape: one target row (get_similar_sets, recommendation_system.py:213-217), one user row (CF,
:438-461), one retriever query with k = 20 (lego_nlp_recommeder.py:305, 1394).

Every case runs both ways on the same index and inputs — the large-batch path (bf16 MFMA scan
+ candidate lists + exact re-rank, BB_OPT_SMALL_BATCH = 0) and the small-batch path (an
approximate f32 pass over the bf16 copy, the candidates within its bound rescored exactly) —
and the lists must be identical bit for bit (ids and score bits); they are also checked
against an f64 recompute over the device's own f32 operands.  Edge cases: ragged batches (every B in 1..16),
k > eligible items, an empty mask, a workgroup holding many of the top items (its list
overflows), masses of equal scores (more than 256 candidates: the exact fallback), rank 0
duplicated, the BB_Q_OUT_KEYS lists of a sharded search, and a tiny index (G5's 10 rows).
"""
import numpy as np
import pytest

from oracle import restatement as R

pytestmark = pytest.mark.gpu

VARIANTS = (0, 1)


@pytest.fixture(scope="module")
def brickrec():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import brickrec as br
    return br


def _qop(q):
    q64 = q.astype(np.float64)
    n = np.sqrt((q64 * q64).sum(1, keepdims=True))
    n[n == 0] = 1.0
    return (q64 / n).astype(np.float32)


def _exact(rows32, q32, k, allowed, drop_present=None):
    s = (rows32.astype(np.float64) @ q32.astype(np.float64)).astype(np.float32)
    ok = allowed.copy()
    if drop_present is not None:
        p = np.where(drop_present, s, -np.inf)
        r0 = int(np.flatnonzero(p == p.max())[0])
        ok[r0] = False
    idx = np.flatnonzero(ok)
    o = np.lexsort((idx, -s[idx]))[:k]
    return idx[o], s[idx[o]]


def _run(idx, variant, *args, **kw):
    idx.set_option("small_batch", variant)
    try:
        return idx.search(*args, **kw)
    finally:
        idx.set_option("small_batch", -1)


def _same(a, b):
    sa, ia, ca = a
    sb, ib, cb = b
    assert np.array_equal(ca, cb), (ca, cb)
    assert np.array_equal(ia, ib)
    assert np.array_equal(sa.view(np.uint32), sb.view(np.uint32))


def _all_variants(idx, *args, **kw):
    outs = [_run(idx, v, *args, **kw) for v in VARIANTS]
    _same(outs[0], outs[1])
    return outs[1]


@pytest.fixture(scope="module")
def c1(brickrec):
    n, d = 25216, 384
    x = R.unit_rows(n, d, 1234)
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x, prenormalized=True)
    rows = idx.get_rows(np.arange(n))
    yield idx, x, rows
    idx.close()


@pytest.mark.parametrize("B", list(range(1, 17)))
def test_semantic_every_batch_size(c1, B):
    idx, x, rows = c1
    k = 10 if B == 1 else 50
    q = R.unit_rows(B, 384, 500 + B) * 3.0  # raw rows: the path normalises them
    sc, ids, cnt = _all_variants(idx, "semantic", k, q_rows=q)
    qn = _qop(q)
    allowed = np.ones(len(rows), bool)
    for b in range(B):
        ri, rs = _exact(rows, qn[b], k, allowed)
        assert list(ids[b]) == list(ri)
        assert np.array_equal(sc[b].view(np.uint32), rs.view(np.uint32))
        assert cnt[b] == k


def test_retriever_k20_and_k128(c1):
    idx, x, rows = c1
    q = R.unit_rows(3, 384, 77)
    for k in (20, 127):  # K_int <= 128: the small-batch bound
        _all_variants(idx, "semantic", k, q_rows=q)


def test_similar_with_mask_rank0_dropped(c1):
    idx, x, rows = c1
    rng = np.random.default_rng(3)
    liked = rng.choice(len(rows), 12, replace=False)
    mask = rng.random(len(rows)) < 0.1
    mask[liked[:6]] = True    # rank 0 (the liked row itself) inside and outside the mask
    mask[liked[6:]] = False
    sc, ids, cnt = _all_variants(idx, "similar", 10, q_items=liked, mask=mask)
    for b, t in enumerate(liked):
        ri, rs = _exact(rows, rows[t], 10, mask, drop_present=np.ones(len(rows), bool))
        assert list(ids[b]) == list(ri)
        assert np.array_equal(sc[b].view(np.uint32), rs.view(np.uint32))


def test_similar_duplicate_rank0(brickrec):
    """A duplicate of the target outranks nothing: ties at rank 0 drop the lower id (the
    arg-max of the (score desc, id asc) order), and the target itself may survive."""
    n, d = 5000, 64
    x = R.unit_rows(n, d, 9)
    x[4321] = x[17]
    x[2000] = x[17]
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x, prenormalized=True)
        rows = idx.get_rows(np.arange(n))
        sc, ids, cnt = _all_variants(idx, "similar", 5, q_items=np.array([4321, 17, 99]))
        for b, t in enumerate((4321, 17, 99)):
            ri, rs = _exact(rows, rows[t], 5, np.ones(n, bool), drop_present=np.ones(n, bool))
            assert list(ids[b]) == list(ri)
    finally:
        idx.close()


def test_cf_rated_excluded(brickrec):
    n, r, B = 25216, 50, 7
    rng = np.random.default_rng(11)
    x = R.unit_rows(n, 384, 5)
    f = rng.normal(0, 0.1, (n, r)).astype(np.float32)
    present = rng.random(n) < 0.9
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x, prenormalized=True)
        idx.upload_cf(f, present=present)
        u = rng.normal(0, 0.1, (B, r)).astype(np.float32)
        rated = np.zeros((B, n), bool)
        for b in range(B):
            rated[b, rng.choice(n, 30, replace=False)] = True
        mask = rng.random(n) < 0.5
        sc, ids, cnt = _all_variants(idx, "cf", 20, q_cf=u, mask=mask, excl=rated)
        f32 = f.astype(np.float32)
        for b in range(B):
            ri, rs = _exact(f32, u[b], 20, mask & present & ~rated[b])
            assert list(ids[b]) == list(ri)
            assert np.array_equal(sc[b].view(np.uint32), rs.view(np.uint32))
    finally:
        idx.close()


@pytest.mark.parametrize("scale", [1e-35, 1e-30])
def test_tiny_query_rows(brickrec, scale):
    """Query rows far below f16 range: the pass scales a row by 2^(14 - e) of its
    largest |q|, the exponent clamped at 126 — 1e-35 rows would otherwise scale to +inf and
    NaN orders.  Raw CF rows (no normalisation) and semantic rows (normalised by the path)."""
    n, r, B = 6000, 50, 5
    rng = np.random.default_rng(31)
    x = R.unit_rows(n, 64, 8)
    f = rng.normal(0, 0.1, (n, r)).astype(np.float32)
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x, prenormalized=True)
        idx.upload_cf(f)
        u = (rng.normal(0, 1.0, (B, r)) * scale).astype(np.float32)
        sc, ids, cnt = _all_variants(idx, "cf", 10, q_cf=u)
        for b in range(B):
            ri, rs = _exact(f, u[b], 10, np.ones(n, bool))
            assert list(ids[b]) == list(ri)
            assert np.array_equal(sc[b].view(np.uint32), rs.view(np.uint32))
        q = (R.unit_rows(B, 64, 9) * scale).astype(np.float32)
        sc, ids, cnt = _all_variants(idx, "semantic", 10, q_rows=q)
        rows = idx.get_rows(np.arange(n))
        qn = _qop(q)
        for b in range(B):
            ri, rs = _exact(rows, qn[b], 10, np.ones(n, bool))
            assert list(ids[b]) == list(ri)
    finally:
        idx.close()


def test_f16_range_saturation(brickrec):
    """Values beyond the f16 range (|x| > 65504) saturate in the approximate copy and in the
    query operands; every bound is computed from the saturated values, so those rows and
    queries only widen the candidate window (here: into the exact slow paths) — both paths
    stay exact.  CF factors with a few huge entries, and one user row with a huge entry."""
    n, r, B = 25216, 50, 4
    rng = np.random.default_rng(12)
    x = R.unit_rows(n, 384, 6)
    f = rng.normal(0, 0.1, (n, r)).astype(np.float32)
    hot = rng.choice(n, 40, replace=False)
    f[hot, rng.integers(0, r, 40)] = rng.choice([-1.0, 1.0], 40) * 2.0e5
    u = rng.normal(0, 0.1, (B, r)).astype(np.float32)
    u[1, 7] = 1.5e5
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x, prenormalized=True)
        idx.upload_cf(f)
        sc, ids, cnt = _all_variants(idx, "cf", 20, q_cf=u)
        for b in range(B):
            ri, rs = _exact(f, u[b], 20, np.ones(n, bool))
            assert list(ids[b]) == list(ri)
            assert np.array_equal(sc[b].view(np.uint32), rs.view(np.uint32))
    finally:
        idx.close()


@pytest.mark.parametrize("B", [1, 3, 16])
def test_hybrid_requests(brickrec, B):
    """HybridRecommender.get_recommendations' shape (recommendation_system.py:612-677): liked set
    + user factors, mask, rated exclusions; both sides' passes, one merge launch for both key
    lists, finalize1's union blend — identical to the large-batch path, and the key lists of a
    sharded hybrid search (BB_Q_OUT_KEYS) identical too."""
    import torch
    n, d, r = 25216, 384, 50
    rng = np.random.default_rng(100 + B)
    x = R.unit_rows(n, d, 1234)
    f = rng.normal(0, 0.1, (n, r)).astype(np.float32)
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x, prenormalized=True)
        idx.upload_cf(f, present=rng.random(n) < 0.8)
        liked = rng.choice(n, B, replace=False)
        u = rng.normal(0, 0.1, (B, r)).astype(np.float32)
        mask = rng.random(n) < 0.2
        rated = rng.random((B, n)) < 0.002
        for k in (10, 50):
            sc, ids, cnt = _all_variants(idx, "hybrid", k, q_items=liked, q_cf=u, mask=mask, excl=rated)
            assert (cnt > 0).all()
        outs = {}
        qi = torch.from_numpy(liked).cuda()
        qc = torch.from_numpy(u).cuda()
        for v in VARIANTS:
            idx.set_option("small_batch", v)
            try:
                outs[v] = idx.search_keys("hybrid", 10, q_items=qi, q_cf=qc)
            finally:
                idx.set_option("small_batch", -1)
        torch.cuda.synchronize()
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    finally:
        idx.close()


def test_k_beyond_eligible_and_empty_mask(c1):
    idx, x, rows = c1
    q = R.unit_rows(2, 384, 8)
    mask = np.zeros(len(rows), bool)
    mask[[5, 900, 25000]] = True
    sc, ids, cnt = _all_variants(idx, "semantic", 10, q_rows=q, mask=mask)
    assert list(cnt) == [3, 3]
    assert (ids[:, 3:] == -1).all() and (sc[:, 3:] == 0).all()
    sc, ids, cnt = _all_variants(idx, "semantic", 10, q_rows=q, mask=np.zeros(len(rows), bool))
    assert list(cnt) == [0, 0] and (ids == -1).all()


def test_overflowed_workgroup_list(brickrec):
    """One workgroup's rows hold the whole top-20 (consecutive near-copies of the query): its
    list of 4 overflows and the merge takes that workgroup's rows from their order images."""
    n, d = 20000, 128
    x = R.unit_rows(n, d, 21)
    q = R.unit_rows(1, d, 22)[0]
    rng = np.random.default_rng(1)
    for i in range(40):
        v = q + 0.02 * rng.standard_normal(d)
        x[3000 + i] = v / np.linalg.norm(v)
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x, prenormalized=True)
        rows = idx.get_rows(np.arange(n))
        sc, ids, cnt = _all_variants(idx, "semantic", 30, q_rows=q[None, :])
        ri, rs = _exact(rows, _qop(q[None, :])[0], 30, np.ones(n, bool))
        assert list(ids[0]) == list(ri)
        assert 3000 <= ids[0][0] < 3040
    finally:
        idx.close()


def test_masses_of_equal_scores_fallback(brickrec):
    """600 identical rows tie at the top: more than 256 candidates reach the bound, so the merge
    runs its slow exact path (batched rescoring into a running top-K); ties resolve by id
    ascending."""
    n, d = 30000, 96
    x = R.unit_rows(n, d, 31)
    q = R.unit_rows(1, d, 32)[0]
    dup = np.sort(np.random.default_rng(2).choice(n, 600, replace=False))
    x[dup] = q
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x, prenormalized=True)
        sc, ids, cnt = _all_variants(idx, "semantic", 100, q_rows=q[None, :])
        assert list(ids[0]) == list(dup[:100])
        assert len(set(sc[0].view(np.uint32))) == 1
    finally:
        idx.close()


def test_out_keys_sharded_lists(c1, brickrec):
    import torch
    idx, x, rows = c1
    q = torch.from_numpy(R.unit_rows(5, 384, 41)).cuda()
    liked = torch.tensor([3, 77, 25000], device="cuda")
    outs = {}
    for v in VARIANTS:
        idx.set_option("small_batch", v)
        try:
            outs[v] = (idx.search_keys("semantic", 50, q_rows=q), idx.search_keys("similar", 10, q_items=liked))
        finally:
            idx.set_option("small_batch", -1)
    torch.cuda.synchronize()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_tiny_index_g5(brickrec):
    n, d = 10, 384
    x = R.unit_rows(n, d, 51)
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x, prenormalized=True)
        sc, ids, cnt = _all_variants(idx, "similar", 3, q_items=np.array([4, 1]))
        rows = idx.get_rows(np.arange(n))
        for b, t in enumerate((4, 1)):
            ri, rs = _exact(rows, rows[t], 3, np.ones(n, bool), drop_present=np.ones(n, bool))
            assert list(ids[b]) == list(ri)
        sc, ids, cnt = _all_variants(idx, "semantic", 20, q_rows=x[:2])
        assert list(cnt) == [10, 10]
    finally:
        idx.close()


def test_device_inputs_and_views(c1, brickrec):
    """Torch device tensors on a view's own stream (the bench's in-flight lanes)."""
    import torch
    idx, x, rows = c1
    v = idx.view()
    try:
        q = torch.from_numpy(R.unit_rows(16, 384, 61)).cuda()
        s = torch.cuda.Stream()
        run, out = v.prepared_search("semantic", 50, q_rows=q, stream=s)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ref = idx.search("semantic", 50, q_rows=q.cpu().numpy())
        assert np.array_equal(out[1].cpu().numpy(), ref[1])
        assert np.array_equal(out[0].cpu().numpy().view(np.uint32), ref[0].view(np.uint32))
    finally:
        v.close()


def test_prepared_search_keeps_its_view_alive(c1):
    """prepared_search's closure holds the index it searches: dropping the last reference to a
    view while its prepared search is still in use must not free the handle under it."""
    import gc
    import torch
    idx, x, rows = c1
    q = torch.from_numpy(R.unit_rows(4, 384, 61)).cuda()
    v = idx.view()
    run, out = v.prepared_search("semantic", 10, q_rows=q)
    del v
    gc.collect()
    run()
    torch.cuda.synchronize()
    ref = idx.search("semantic", 10, q_rows=q.cpu().numpy())
    assert np.array_equal(out[1].cpu().numpy(), ref[1])
    del run
    gc.collect()


def _torch_args(dev, **kw):
    import torch
    out = {}
    for k, v in kw.items():
        if v is None:
            continue
        if k in ("mask", "excl"):
            v = torch.from_numpy(np.asarray(v).view(np.int32) if np.asarray(v).dtype == np.uint32
                                 else __import__("brickrec").bits_from_bool(v).view(np.int32))
        else:
            v = torch.from_numpy(np.ascontiguousarray(v))
        out[k] = v.to(dev)
    return out


@pytest.mark.parametrize("B", [1, 16, 256])
def test_plan_replays_the_search(brickrec, B):
    """prepared_search runs a bb_plan — the host side of the search ran once,
    each call replays its launches on the inputs' CURRENT contents.  Every mode (semantic,
    similar with a mask, CF with rated exclusions, hybrid), on the small-batch (B <= 16) and the
    list (B = 256) paths: the replayed results equal bb_search's bit for bit after the query
    buffers are rewritten in place between calls."""
    import torch
    dev = torch.device("cuda", 0)
    n, d, r = 25216, 384, 50
    rng = np.random.default_rng(900 + B)
    x = R.unit_rows(n, d, 1234)
    f = rng.normal(0, 0.1, (n, r)).astype(np.float32)
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x, prenormalized=True)
        idx.upload_cf(f)
        mask = rng.random(n) < 0.3
        excl = rng.random((B, n)) < 0.002
        cases = {"semantic": dict(q_rows=R.unit_rows(B, d, 5)),
                 "similar": dict(q_items=rng.choice(n, B, replace=False).astype(np.int64), mask=mask),
                 "cf": dict(q_cf=rng.normal(0, 0.1, (B, r)).astype(np.float32), excl=excl),
                 "hybrid": dict(q_items=rng.choice(n, B, replace=False).astype(np.int64),
                                q_cf=rng.normal(0, 0.1, (B, r)).astype(np.float32), mask=mask, excl=excl)}
        for mode, kw in cases.items():
            k = 10
            targs = _torch_args(dev, **kw)
            run, out = idx.prepared_search(mode, k, **targs)
            assert type(run).__name__ == "_Plan", type(run)
            for rep in range(3):
                if rep:   # new request contents in the same buffers
                    if "q_rows" in kw:
                        kw["q_rows"] = R.unit_rows(B, d, 50 + rep)
                    if "q_items" in kw:
                        kw["q_items"] = rng.choice(n, B, replace=False).astype(np.int64)
                    if "q_cf" in kw:
                        kw["q_cf"] = rng.normal(0, 0.1, (B, r)).astype(np.float32)
                    for key in ("q_rows", "q_items", "q_cf"):
                        if key in kw:
                            targs[key].copy_(torch.from_numpy(kw[key]).to(dev))
                run()
                torch.cuda.synchronize()
                ref = idx.search(mode, k, **kw)
                assert np.array_equal(out[2].cpu().numpy(), ref[2]), (mode, rep)
                assert np.array_equal(out[1].cpu().numpy(), ref[1]), (mode, rep)
                assert np.array_equal(out[0].cpu().numpy().view(np.uint32), ref[0].view(np.uint32)), (mode, rep)
            # while the plan lives the index takes no upload (its private view reads the rows)
            with pytest.raises(brickrec.BrickrecError):
                idx.upload_cf(f)
            run.close()
        idx.upload_cf(f)   # every plan closed: uploads work again
    finally:
        idx.close()


def test_plan_refused_on_streaming_falls_back(brickrec):
    """A streaming search reads its overflow flag on the host: bb_plan_create refuses it
    (BB_E_HOSTSYNC, a code of its own: ADVICE r05) and prepared_search keeps the bb_search
    call — same results, and run.is_plan says so."""
    import torch
    n, d, B, k = 3000, 128, 40, 10      # B > 16: not the small-batch path
    x = R.unit_rows(n, d, 31)
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x)
        idx.set_option("stream", 1)
        q = torch.from_numpy(R.unit_rows(B, d, 32)).cuda()
        run, out = idx.prepared_search("semantic", k, q_rows=q)
        assert type(run).__name__ != "_Plan" and run.is_plan is False
        run()
        torch.cuda.synchronize()
        ref = idx.search("semantic", k, q_rows=q.cpu().numpy())
        assert np.array_equal(out[1].cpu().numpy(), ref[1])
    finally:
        idx.close()


def test_destroyed_handle_is_an_error(brickrec):
    """VERDICT r04 item 6 on the device: a handle already passed to bb_destroy (the r04r
    use-after-free) returns BB_E_ARG from bb_search, and a closed plan from bb_plan_launch."""
    import ctypes as C
    import torch
    from brickrec import _lib as L
    lib = L.load()
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(R.unit_rows(1000, 64, 3))
    q = torch.from_numpy(R.unit_rows(2, 64, 4)).cuda()
    run, out = idx.prepared_search("semantic", 5, q_rows=q)
    p = run._p
    h = C.c_void_p(idx._h.value)
    idx.close()          # closes the plan first, then the index
    assert lib.bb_plan_launch(p) == L.BB_E_ARG
    qs = L.bb_query(mode=L.BB_MODE_SEMANTIC, B=2, k=5, where=L.BB_DEVICE, q_rows=q.data_ptr())
    res = L.bb_result(scores=out[0].data_ptr(), ids=out[1].data_ptr(), where=L.BB_DEVICE)
    assert lib.bb_search(h, C.byref(qs), C.byref(res)) == L.BB_E_ARG
    assert b"stale or foreign" in lib.bb_last_error()
    assert lib.bb_destroy(h) == L.BB_E_ARG


def test_plan_launched_from_two_threads(brickrec):
    """bb_plan_launch holds the plan's lock while it enqueues, so two
    threads replaying ONE plan never interleave their launches on its workspace.  Both threads
    replay the list-path plan (B = 256: prep -> scan -> select, three dependent launches over
    shared scratch) 40 times each; the results equal bb_search's bit for bit.  Then a second
    destroy of the same plan is an error, not a double free."""
    import ctypes as C
    import threading
    import torch
    from brickrec import _lib as L
    dev = torch.device("cuda", 0)
    n, d, B, k = 25216, 384, 256, 50
    x = R.unit_rows(n, d, 77)
    qn = R.unit_rows(B, d, 78)
    idx = brickrec.ItemIndex(dtype="f32")
    try:
        idx.upload_items(x, prenormalized=True)
        q = torch.from_numpy(qn).to(dev)
        run, out = idx.prepared_search("semantic", k, q_rows=q)
        assert run.is_plan
        errs = []

        def worker():
            try:
                for _ in range(40):
                    run()
            except Exception as e:   # pragma: no cover - reported below
                errs.append(e)
        ts = [threading.Thread(target=worker) for _ in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        torch.cuda.synchronize()
        assert not errs, errs
        ref = idx.search("semantic", k, q_rows=qn)
        assert np.array_equal(out[1].cpu().numpy(), ref[1])
        assert np.array_equal(out[0].cpu().numpy().view(np.uint32), ref[0].view(np.uint32))
        lib = L.load()
        p = run._p
        run.close()
        assert lib.bb_plan_destroy(p) == L.BB_E_ARG      # already destroyed
        assert b"stale or foreign" in lib.bb_last_error()
    finally:
        idx.close()
