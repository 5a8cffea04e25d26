"""Pin the oracle: oracle/restatement.py vs the golden vectors the reference itself produced
(oracle/gen_golden.py ran src/scripts/recommendation_system.py and
hard_constraint_filter.py in the build container; G5 holds the reference's own MiniLM
vectors from test_embeddings/).  CPU only.

Bar: ids exact (order included), scores within 1e-5 (fp32 summation-order noise).
"""
import hashlib
import json

import numpy as np
import pytest

from oracle import restatement as R
from _spaces import catalog_json, constraint_pairs, hybrid_space

TOL = 1e-5


def _eq(ids, scores, ref_ids, ref_scores, tol=TOL):
    ids = np.asarray(ids)
    ref_ids = np.asarray(ref_ids)
    assert list(ids) == list(ref_ids), f"ids differ:\n{ids}\n{ref_ids}"
    np.testing.assert_allclose(np.asarray(scores, np.float64), ref_scores, atol=tol, rtol=0)


# --------------------------------------------------------------------- G1 content similar
def test_g1_similar_sets(golden):
    g = golden("g1_content.npz")
    x, k = g["feat_matrix"], int(g["k"])
    for i, q in enumerate(g["query_rows"]):
        ids, sc = R.similar_sets(x, int(q), k)
        _eq(ids, sc, g["ids_nofilter"][i], g["scores_nofilter"][i])
        ids, sc = R.similar_sets(x, int(q), k, g["filter_mask"])
        _eq(ids, sc, g["ids_filter"][i], g["scores_filter"][i])


def test_g1_filter_mask_is_the_restated_predicate(golden):
    """The G1 valid filter (pieces <= 800 and year >= 2005) through constraint_mask."""
    g, g4 = golden("g1_content.npz"), golden("g4_hybrid.npz")
    cat = R.Catalog(g["num_parts"], g["year"], g["theme_id"])
    m = R.constraint_mask(cat, [("pieces_max", 800), ("year_min", 2005)], int(g4["current_year"]))
    assert np.array_equal(m, g["filter_mask"])


def test_g1_rank0_is_argmax_not_query(golden):
    """Rank 0 dropped by the reference is the arg-max of the row (itself in these rows)."""
    g = golden("g1_content.npz")
    x = g["feat_matrix"]
    for q in g["query_rows"]:
        sim = R.cosine_scores(x[int(q):int(q) + 1], x)[0]
        r0 = R.rank0(sim)
        assert sim[r0] == sim.max()
        assert r0 not in g["ids_nofilter"][list(g["query_rows"]).index(q)]


# --------------------------------------------------------------------- G2 384-d vectors
def test_g2_semantic_and_similar(golden):
    g = golden("g2_semantic.npz")
    x = R.unit_rows(int(g["n_items"]), 384, 1234)
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["items_sha256"])
    k = int(g["k"])
    ids, sc = R.semantic_topk(x, g["queries"], k)
    for i in range(len(ids)):
        _eq(ids[i], sc[i], g["semantic_ids"][i], g["semantic_scores"][i])
    for i, q in enumerate(g["similar_rows"]):
        ids, sc = R.similar_sets(x, int(q), k)
        _eq(ids, sc, g["similar_ids"][i], g["similar_scores"][i])


# --------------------------------------------------------------------- G5 reference MiniLM
def test_g5_minilm_known_answer(golden):
    g = golden("g5_faiss.npz")
    x = g["vectors"]
    n = x.shape[0]
    for i in range(n):
        ids, sc = R.similar_sets(x, i, n - 1)
        _eq(ids, sc, g["ids"][i], g["scores"][i])
    names = list(g["set_nums"])
    i = names.index("75192-1")
    ids, sc = R.similar_sets(x, i, 3)
    assert [names[j] for j in ids] == ["75331-1", "75313-1", "10294-1"]
    assert abs(sc[0] - 0.845918) < 1e-5


# --------------------------------------------------------------------- G3 CF
def test_g3_cf(golden):
    g = golden("g3_cf.npz")
    users = list(g["user_ids"])
    k2 = 2 * int(g["k"])
    for i, u in enumerate(g["query_users"]):
        r = users.index(u)
        ids, sc = R.cf_topk(g["user_factors"][r], g["item_factors"], k2, rated=g["rated"][r])
        L = int(g["lens"][i])
        _eq(ids[:L], sc[:L], g["ids"][i][:L], g["scores"][i][:L])


# --------------------------------------------------------------------- G4 masks + hybrid
def test_g4_constraint_masks(golden):
    g1, g4 = golden("g1_content.npz"), golden("g4_hybrid.npz")
    cat = catalog_json()
    themes = {int(k): v for k, v in cat["themes"].items()}
    c = R.Catalog(g1["num_parts"], g1["year"], g1["theme_id"], themes,
                  owned={3: set(int(i) for i in g4["owned_rows"])},
                  wishlisted={3: set(int(i) for i in g4["wished_rows"])})
    for ci, cj in enumerate(g4["case_json"]):
        kw = json.loads(str(cj))
        pairs = constraint_pairs(kw)
        pairs = [(t, 3 if t.startswith("exclude_") else v) for t, v in pairs]
        m = R.constraint_mask(c, pairs, int(g4["current_year"]))
        assert np.array_equal(m, g4["masks"][ci]), f"case {ci} {kw}"


def test_g4_hybrid(golden):
    g4, g3 = golden("g4_hybrid.npz"), golden("g3_cf.npz")
    X, present, F, cf_present, rated, n, n_rows = hybrid_space(golden)
    users = list(g3["user_ids"])
    k = int(g4["k"])
    for case, (u, qrow, ci) in enumerate(g4["hybrid_meta"]):
        allowed = np.ones(n, bool)
        if ci >= 0:
            allowed[:] = False
            allowed[:n_rows] = g4["masks"][ci]
        c_i = c_s = f_i = f_s = np.zeros(0)
        if qrow >= 0:
            c_i, c_s = R.similar_sets(X, int(qrow), 2 * k, allowed & present)
        if u >= 0:
            r = users.index(u)
            f_i, f_s = R.cf_topk(g3["user_factors"][r], F, 2 * k, allowed, rated[r], cf_present)
        if len(c_i) and len(f_i):
            ids, sc = R.union_blend(c_i, c_s, f_i, f_s, 0.4, 0.6, k)
        elif len(c_i):
            ids, sc = c_i[:k], c_s[:k]
        else:
            ids, sc = f_i[:k], f_s[:k]
        L = int(g4["lens"][case])
        assert len(ids) == L
        _eq(ids, sc, g4["ids"][case][:L], g4["scores"][case][:L])


# --------------------------------------------------------------------- oracle internals
def test_topk_tie_rule_and_ragged():
    s = np.array([0.5, 0.9, 0.5, 0.9, 0.1], np.float32)
    ids, sc = R.topk_indices(s, 3)
    assert list(ids) == [1, 3, 0]
    ids, sc = R.topk_indices(s, 10, np.array([1, 0, 1, 0, 0], bool))
    assert list(ids) == [0, 2]
    ids, sc = R.topk_indices(s, 0)
    assert ids.size == 0
    ids, sc = R.topk_indices(s, 3, np.zeros(5, bool))
    assert ids.size == 0


def test_zero_rows_score_zero():
    x = np.array([[1.0, 0.0], [0.0, 0.0], [0.6, 0.8]])
    sim = R.cosine_scores(x[:1], x)[0]
    assert sim[1] == 0.0 and abs(sim[0] - 1.0) < 1e-12


def test_union_blend_missing_side_scores_zero():
    ids, sc = R.union_blend([1, 2], [0.9, 0.5], [2, 3], [1.0, 0.2], 0.4, 0.6, 3)
    # h(1) = 0.36, h(2) = 0.2 + 0.6 = 0.8, h(3) = 0.12
    assert list(ids) == [2, 1, 3]
    np.testing.assert_allclose(sc, [0.8, 0.36, 0.12])


def test_batched_cosine_topk_matches_semantic():
    x = R.unit_rows(3000, 64, 7)
    q = R.unit_rows(8, 64, 8)
    bi, bs = R.batched_cosine_topk(x, q, 20)
    si, ss = R.semantic_topk(x, q, 20)
    for i in range(8):
        assert list(bi[i]) == list(si[i])
        np.testing.assert_allclose(bs[i], ss[i], atol=1e-6)
