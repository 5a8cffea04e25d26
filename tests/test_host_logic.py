"""Host-side logic of the drop-in, CPU only: bitset packing, the constraint -> Predicate
compiler (checked against the reference's own apply_constraints masks in G4 through a
numpy evaluation of the Predicate with the mask kernel's semantics), LIKE matching and the
reference's constraint helper functions."""
import json

import numpy as np
import pytest

from _spaces import catalog_json
from brickrec.constraints import (ConstraintType, HardConstraint, create_age_appropriate_constraints,
                                  create_budget_constraints, create_constraint_set_values,
                                  create_size_constraints, predicate_from_constraints, theme_ids_like)
from brickrec.engine import INT32_MAX, INT32_MIN, Predicate, bits_from_bool, bool_from_bits


def eval_predicate(p: Predicate, parts, year, theme, n_ids=None):
    """numpy statement of mask_kernel (csrc/misc.hip): inclusive bounds, num_parts > 0,
    theme tests with SQL NULL (theme < 0) -> false, then excluded ids cleared."""
    parts, year, theme = (np.asarray(a, np.int64) for a in (parts, year, theme))
    m = (parts > 0) & (parts >= p.parts_min) & (parts <= p.parts_max)
    m &= (year >= p.year_min) & (year <= p.year_max)
    if p.theme_mode:
        inset = np.isin(theme, list(p.theme_ids))
        m &= (theme >= 0) & (inset if p.theme_mode == 1 else ~inset)
    if len(p.excluded_items):
        m[np.asarray(p.excluded_items, np.int64)] = False
    return m


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 1000])
def test_bits_round_trip(n):
    rng = np.random.default_rng(n)
    m = rng.random(n) < 0.3
    w = bits_from_bool(m)
    assert w.dtype == np.uint32 and w.shape == ((n + 31) // 32,)
    assert np.array_equal(bool_from_bits(w, n), m)
    for i in np.flatnonzero(m):
        assert (w[i // 32] >> (i % 32)) & 1


def test_bits_batched():
    m = np.zeros((3, 70), bool)
    m[1, 69] = m[2, 0] = True
    w = bits_from_bool(m)
    assert w.shape == (3, 3)
    assert w[1, 2] == 1 << 5 and w[2, 0] == 1


def test_predicate_compiler_matches_reference_masks(golden):
    g1, g4 = golden("g1_content.npz"), golden("g4_hybrid.npz")
    cat = catalog_json()
    themes = {int(k): v for k, v in cat["themes"].items()}
    owned = {3: set(int(i) for i in g4["owned_rows"])}
    wished = {3: set(int(i) for i in g4["wished_rows"])}
    for ci, cj in enumerate(g4["case_json"]):
        kw = json.loads(str(cj))
        pred = predicate_from_constraints(create_constraint_set_values(**kw), themes, owned, wished,
                                          int(g4["current_year"]))
        if pred is None:
            m = np.zeros(len(g1["num_parts"]), bool)
        else:
            m = eval_predicate(pred, g1["num_parts"], g1["year"], g1["theme_id"])
        assert np.array_equal(m, g4["masks"][ci]), f"case {ci} {kw}"


def test_predicate_int32_ranges():
    p = predicate_from_constraints([], {}, {}, {}, 2025)
    assert (p.parts_min, p.parts_max, p.year_min, p.year_max) == (INT32_MIN, INT32_MAX, INT32_MIN, INT32_MAX)
    p = predicate_from_constraints(create_constraint_set_values(price_max=45.0, pieces_max=300), {}, {}, {}, 2025)
    assert p.parts_max == 300
    p = predicate_from_constraints(create_constraint_set_values(price_max=45.0, pieces_max=900), {}, {}, {}, 2025)
    assert p.parts_max == int(45.0 / 0.10)
    p = predicate_from_constraints(create_constraint_set_values(must_be_available=True), {}, {}, {}, 2025)
    assert p.year_min == 2020


def test_required_and_excluded_themes_combine():
    names = {1: "Star Wars", 2: "Star Wars Ultimate", 3: "City", 4: "Technic"}
    c = create_constraint_set_values(required_themes=["star wars"], excluded_themes=["ultimate"])
    p = predicate_from_constraints(c, names, {}, {}, 2025)
    assert p.theme_mode == 1 and list(p.theme_ids) == [1]
    c = create_constraint_set_values(excluded_themes=["city", "zzz"])
    p = predicate_from_constraints(c, names, {}, {}, 2025)
    assert p.theme_mode == 2 and list(p.theme_ids) == [3]
    assert predicate_from_constraints(create_constraint_set_values(required_themes=["zzz"]),
                                      names, {}, {}, 2025) is None


def test_like_semantics():
    names = {1: "Star Wars", 2: "Harry_Potter", 3: "100% Fun", 4: "Space"}
    assert theme_ids_like(names, ["STAR"]) == [1]
    assert theme_ids_like(names, ["y_p"]) == [2]          # '_' matches one character
    assert theme_ids_like(names, ["0%f"]) == [3]          # '%' matches any run
    assert theme_ids_like(names, ["a"]) == [1, 2, 4]


def test_constraint_helpers():
    b = create_budget_constraints(100.0, 20.0)
    assert [c.constraint_type for c in b] == [ConstraintType.PRICE_MAX, ConstraintType.PRICE_MIN]
    a = create_age_appropriate_constraints(10)
    assert a[0].constraint_type == ConstraintType.AGE_MIN and a[0].value == 8
    assert create_age_appropriate_constraints(5, strict=False)[0].value == 4
    s = create_size_constraints("Medium")
    assert [(c.constraint_type, c.value) for c in s] == [(ConstraintType.PIECES_MIN, 201),
                                                         (ConstraintType.PIECES_MAX, 800)]
    assert create_size_constraints("huge") == []
    h = HardConstraint(ConstraintType.PIECES_MAX, 10)
    assert h.description == "pieces_max: 10"


def test_blend_sure_is_sound_and_tight():
    """tests/_parity.blend_sure (the configs[2] near-tie membership check): with clear side
    boundaries it names the oracle's whole blended top-k (minus final-boundary near-ties);
    with a side boundary forced into a tie it names only items whose membership cannot change,
    and each of those is in the blend under either resolution of the tie."""
    import numpy as np
    from oracle import restatement as R
    from _parity import blend_sure
    rng = np.random.default_rng(3)
    for trial in range(40):
        n, ks, k = 400, 20, 10
        c = rng.normal(0, 1, n)
        f = rng.normal(0, 1, n)
        if trial % 2:          # force a near-tie at the content boundary
            o = np.argsort(-c)
            c[o[ks]] = c[o[ks - 1]] - 1e-7
        ci, cs = R.topk_indices(c, ks + 8)
        fi, fs = R.topk_indices(f, ks + 8)
        sure = blend_sure(ci, cs, fi, fs, ks, 0.4, 0.6, k)
        # both resolutions of a content-boundary tie: the ks-th or the (ks+1)-th item in the list
        for swap in ((False, True) if trial % 2 else (False,)):
            cl, csl = list(ci[:ks]), list(cs[:ks])
            if swap:
                cl[-1], csl[-1] = ci[ks], cs[ks]
            hi, hs = R.union_blend(cl, csl, fi[:ks], fs[:ks], 0.4, 0.6, k)
            got = dict(zip(hi.tolist(), hs.tolist()))
            for i, h in sure.items():
                assert i in got and abs(got[i] - h) < 1e-12
        if trial % 2 == 0:
            assert len(sure) >= k - 2


def test_constraint_first_equivalence():
    """DESIGN §3a'' (compact.hip), the argument on the CPU oracle: searching only the rows the
    mask allows — packed in ascending id order at slot p·stride, the liked set's rank-0 item
    (the arg-max of the UNMASKED ranking, recommendation_system.py:217, from a per-item table)
    excluded when it is allowed, ties by slot — gives exactly get_similar_sets' masked list,
    and the CF and hybrid lists too.  Duplicate rows make rank 0 another id (and an allowed
    one); masks from 0 to all rows; strides 1, 2 and 4."""
    from oracle import restatement as R
    rng = np.random.default_rng(11)
    n, d, r, k = 600, 16, 4, 7
    x = rng.standard_normal((n, d)).astype(np.float32)
    x[[50, 90, 400]] = x[20]                 # rank 0 of 50 / 90 / 400 is 20 (lowest id of the twins)
    f = (0.1 * rng.standard_normal((n, r))).astype(np.float32)
    # the oracle's own scores, row by row as get_similar_sets computes them: the argument is
    # about which rows are searched, not about arithmetic
    sims = np.stack([R.cosine_scores(x[i:i + 1], x)[0] for i in range(n)])
    r0_table = np.array([R.rank0(sims[i]) for i in range(n)])      # the upload-time table
    for density in (0.0, 0.02, 0.3, 1.0):
        mask = rng.random(n) < density
        mask[[20, 50]] = density > 0
        allowed = np.flatnonzero(mask)
        for stride in (1, 2, 4):
            slots = np.full(max(len(allowed), 1) * stride, -1, np.int64)
            slots[::stride][:len(allowed)] = allowed                 # slot -> id (idmap)
            real = slots >= 0
            for liked in (20, 50, 90, 7, 599):
                want_i, want_s = R.similar_sets(x, liked, k, mask)
                s = np.where(real, sims[liked][np.maximum(slots, 0)], -np.inf)
                ok = real.copy()
                r0 = r0_table[liked]
                if mask[r0]:
                    ok[np.flatnonzero(slots == r0)] = False          # the content exclusion bit
                got_slot, got_s = R.topk_indices(s, k, ok)
                assert list(slots[got_slot]) == list(want_i), (density, stride, liked)
                assert np.array_equal(got_s, want_s)
            u = (0.1 * rng.standard_normal(r)).astype(np.float32)
            rated = rng.random(n) < 0.05
            want_i, _ = R.cf_topk(u, f, k, mask, rated)
            fs = np.where(real, (f @ u)[np.maximum(slots, 0)], -np.inf)
            got_slot, _ = R.topk_indices(fs, k, real & ~rated[np.maximum(slots, 0)])
            assert list(slots[got_slot]) == list(want_i)


def test_finalize_pruned_rank_equals_full_rank():
    """finalize_body.h's ranking, restated on the host: the pruning bound T (the k-th largest
    f32 image among a sample of the entries) drops only entries that rank >= k, and the
    survivors' ranks — the count of strictly larger images, plus, where the claim table finds
    a shared count, the (h desc, id asc) comparison among equal images — equal their ranks
    among all entries.  Heavy ties (h rounded to a coarse grid, duplicate f32 images of
    distinct f64 h) and every sample size around k."""
    rng = np.random.default_rng(5)
    for trial in range(300):
        n = int(rng.integers(1, 220))
        k = int(rng.integers(1, 80))
        h = rng.normal(0.0, 0.2, n)
        if trial % 3 == 0:
            h = np.round(h * 16) / 16                      # exact ties
        if trial % 3 == 1:
            h = h.astype(np.float32).astype(np.float64) + rng.integers(0, 2, n) * 1e-12  # equal f32, distinct f64
        h = h + 0.0   # (no -0.0: the device's scores are +0-folded, rr_key, so no blend is -0.0)
        g = rng.permutation(100000)[:n].astype(np.int64)   # ids
        img = np.float32(h).view(np.uint32)
        img = np.where(img & 0x80000000, ~img, img | 0x80000000).astype(np.uint64)   # ord_of
        true_order = sorted(range(n), key=lambda e: (-h[e], g[e]))
        true_rank = np.empty(n, int)
        true_rank[true_order] = np.arange(n)
        ns = int(min(n, rng.integers(0, 70)))
        samp = rng.choice(n, ns, replace=False)
        T = 0
        if ns >= k:
            T = int(np.sort(img[samp])[::-1][k - 1])
        surv = np.flatnonzero(img >= T)
        assert np.all(true_rank[img < T] >= k)
        gt = np.array([(img[surv] > img[e]).sum() for e in surv])
        claim = np.bincount(gt, minlength=len(surv) + 1)
        for j, e in enumerate(surv):
            r = gt[j]
            if claim[gt[j]] > 1:
                same = surv[img[surv] == img[e]]
                r += sum(1 for x in same if h[x] > h[e] or (h[x] == h[e] and g[x] < g[e]))
            assert r == true_rank[e], (trial, e)
