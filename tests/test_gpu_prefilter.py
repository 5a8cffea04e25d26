"""Constraint-first search (compact.hip, BB_OPT_PREFILTER): a selective mask's allowed rows are
packed and only they are searched — the reference's "apply hard constraints first"
(recommendation_system.py:628-656).  Every case runs the same search with the prefilter forced
on and off and asserts identical bits (ids, scores, counts), and checks that the packed path
actually ran (one "pack"-family launch: the packing kernel, which also runs the query prep).

Cases: every mode (semantic, similar with rank-0 inside and outside the mask, CF with rated
exclusions, hybrid), masks of 0.1 % .. 25 %, an empty mask, exact duplicates of liked rows (the
rank-0 item is another id), an id outside the index (zero query row), B = 17 .. 1,024, the
torch path with a device mask and its count, a prepared plan, and a device count below the
true count (documented: empty results, never a wrong list).
"""
import numpy as np
import pytest

from oracle import restatement as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def brickrec():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import brickrec as br
    return br


@pytest.fixture(scope="module")
def index(brickrec):
    n, d, r = 25216, 384, 50
    rng = np.random.default_rng(606)
    x = R.unit_rows(n, d, 607)
    x[[5000, 9000, 12000]] = x[3000]          # exact duplicates: rank 0 of 3000 is id 3000's lowest twin
    f = rng.normal(0.0, 0.1, (n, r)).astype(np.float32)
    present = np.ones(n, bool)
    present[rng.choice(n, 50, replace=False)] = False   # rows outside the CF item space
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    idx.upload_cf(f, present=present)
    yield idx, n, r, rng
    idx.close()


def _both(idx, mode, k, **kw):
    out = {}
    for opt in (0, 1):
        idx.set_option("prefilter", opt)
        idx.set_profiling(True)
        out[opt] = idx.search(mode, k, **kw)
        prof = idx.profile()
        idx.set_profiling(False)
        out[f"pack{opt}"] = prof["pack"]["launches"]
    idx.set_option("prefilter", -1)
    return out


def _same(o, B):
    (s0, i0, c0), (s1, i1, c1) = o[0], o[1]
    assert np.array_equal(c0, c1), (c0[:8], c1[:8])
    assert np.array_equal(i0, i1), np.flatnonzero((i0 != i1).any(1))[:8]
    assert np.array_equal(s0.view(np.uint32), s1.view(np.uint32))
    assert (o["pack0"], o["pack1"]) == (0, 1), (o["pack0"], o["pack1"])   # the packing kernel ran


@pytest.mark.parametrize("density", [0.001, 0.0175, 0.1, 0.25])
@pytest.mark.parametrize("mode", ["semantic", "similar", "cf", "hybrid"])
def test_prefilter_identical(index, mode, density):
    idx, n, r, rng = index
    B, k = 256, 20
    mask = rng.random(n) < density
    kw = {"mask": mask}
    if mode == "semantic":
        kw["q_rows"] = R.unit_rows(B, 384, 11)
    if mode in ("similar", "hybrid"):
        liked = rng.choice(n, B, replace=False)
        allowed = np.flatnonzero(mask)
        liked[: min(20, len(allowed))] = allowed[:20]       # rank 0 inside the mask
        liked[20:24] = [3000, 5000, 9000, 12000]            # duplicated rows
        liked[24] = n + 7                                   # outside the index: a zero row
        kw["q_items"] = liked
    if mode in ("cf", "hybrid"):
        kw["q_cf"] = rng.normal(0.0, 0.1, (B, r)).astype(np.float32)
        kw["excl"] = rng.random((B, n)) < 0.002
    _same(_both(idx, mode, k, **kw), B)


@pytest.mark.parametrize("B", [17, 1024])
def test_prefilter_batch_sizes_and_empty_mask(index, B):
    idx, n, r, rng = index
    liked = rng.choice(n, B, replace=False)
    u = rng.normal(0.0, 0.1, (B, r)).astype(np.float32)
    mask = rng.random(n) < 0.02
    _same(_both(idx, "hybrid", 50, q_items=liked, q_cf=u, mask=mask, excl=rng.random((B, n)) < 0.001), B)
    empty = np.zeros(n, bool)
    o = _both(idx, "similar", 10, q_items=liked, mask=empty)
    _same(o, B)
    assert (o[1][2] == 0).all() and (o[1][1] == -1).all()


def test_prefilter_torch_device_mask_and_plan(index, brickrec):
    """The serving shape: a device bitset with its count (bb_query.mask_count), through
    bb_search and through a prepared plan, equals the full search."""
    import torch
    idx, n, r, rng = index
    dev = torch.device("cuda", 0)
    B, k = 512, 50
    mask = rng.random(n) < 0.03
    liked = rng.choice(n, B, replace=False)
    u = rng.normal(0.0, 0.1, (B, r)).astype(np.float32)
    rated = rng.random((B, n)) < 0.001
    idx.set_option("prefilter", 0)
    ref = idx.search("hybrid", k, q_items=liked, q_cf=u, mask=mask, excl=rated)
    idx.set_option("prefilter", -1)
    mw = torch.from_numpy(brickrec.bits_from_bool(mask).view(np.int32)).to(dev)
    ew = torch.from_numpy(brickrec.bits_from_bool(rated).view(np.int32)).to(dev)
    args = dict(q_items=torch.from_numpy(liked).to(dev), q_cf=torch.from_numpy(u).to(dev), mask=mw, excl=ew,
                mask_count=int(mask.sum()))
    got = idx.search("hybrid", k, **args)
    torch.cuda.synchronize()
    for a, b in zip(got, ref):
        assert np.array_equal(a.cpu().numpy(), b)
    run, out = idx.prepared_search("hybrid", k, **args)
    assert run.is_plan
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    assert np.array_equal(out[1].cpu().numpy(), ref[1])
    assert np.array_equal(out[0].cpu().numpy().view(np.uint32), ref[0].view(np.uint32))
    run.close()
    # a device count below the true count: empty results, never a wrong list
    bad = idx.search("hybrid", k, **dict(args, mask_count=max(1, int(mask.sum()) // 3)))
    torch.cuda.synchronize()
    assert (bad[2].cpu().numpy() == 0).all()
