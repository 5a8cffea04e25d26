"""Drop-in parity checks shared by the CPU run (OracleIndex stand-in) and the GPU run (the
HIP ItemIndex): the reference's synthetic sqlite catalogue is rebuilt bit-identically
(oracle/gen_golden.py's builders: same seeds, no reference code involved). The drop-in
classes run over it and must reproduce the reference's own outputs stored in
tests/golden (G1 content + reasons, G3 CF, G4 masks + hybrid).
"""
import json

import numpy as np

from _spaces import catalog_json

TOL = 1e-5


class _DictRows:  # sentinel for PgOnSqlite's RealDictCursor slot
    pass


def build_world():
    from oracle.gen_golden import PgOnSqlite, build_catalog, make_db
    themes, sets, invs, iparts = build_catalog()
    rng = np.random.default_rng(11)
    owned = [(3, sets[int(i)][0]) for i in rng.choice(len(sets), 60, replace=False)]
    wished = [(3, sets[int(i)][0]) for i in rng.choice(len(sets), 40, replace=False)]
    db = make_db(themes, sets, invs, iparts, owned, wished)
    return PgOnSqlite(db, _DictRows)


def pin_year(monkeypatch):
    import brickrec.recommenders as RS
    year = int(catalog_json()["generated_year"])
    monkeypatch.setattr(RS, "_current_year", lambda: year)


def make_hybrid(conn, index_factory):
    from brickrec.catalog import Engine
    from brickrec.recommenders import HybridRecommender
    return HybridRecommender(conn, Engine(conn, index_factory=index_factory))


def _eq_lists(got_ids, got_sc, ref_ids, ref_sc):
    assert list(got_ids) == list(ref_ids), f"ids differ:\n{list(got_ids)}\n{list(ref_ids)}"
    np.testing.assert_allclose(np.asarray(got_sc, np.float64), ref_sc, atol=TOL, rtol=0)


def check_features(hy, golden):
    cb = hy.content_recommender
    cb.prepare_features()
    g1 = golden("g1_content.npz")
    np.testing.assert_array_equal(cb.feat_matrix.astype(np.float64), g1["feat_matrix"])


def check_similar_sets(hy, golden):
    cb = hy.content_recommender
    if cb.feat_matrix is None:
        cb.prepare_features()
    g1 = golden("g1_content.npz")
    cat = catalog_json()
    rows = cat["row_set_nums"]
    pos = {s: i for i, s in enumerate(rows)}
    k = int(g1["k"])
    filt = [s for s, m in zip(rows, g1["filter_mask"]) if m]
    for qi, q in enumerate(g1["query_rows"]):
        recs = cb.get_similar_sets(rows[int(q)], k)
        _eq_lists([pos[r.set_num] for r in recs], [r.score for r in recs],
                  g1["ids_nofilter"][qi], g1["scores_nofilter"][qi])
        assert [r.reasons for r in recs] == cat["g1_reasons_nofilter"][qi]
        for r in recs:
            i = pos[r.set_num]
            assert (r.name, r.img_url, r.theme_name) == (cat["names"][i], cat["img_urls"][i], cat["theme_names"][i])
        recs = cb.get_similar_sets(rows[int(q)], k, valid_set_filter=filt)
        _eq_lists([pos[r.set_num] for r in recs], [r.score for r in recs],
                  g1["ids_filter"][qi], g1["scores_filter"][qi])
    assert cb.get_similar_sets("no-such-set", 5) == []


def check_cf(hy, golden):
    cf = hy.collaborative_recommender
    cf.train_svd_model()
    g3 = golden("g3_cf.npz")
    np.testing.assert_allclose(cf.user_factors, g3["user_factors"], atol=1e-12, rtol=0)
    np.testing.assert_allclose(cf.item_factors, g3["item_factors"], atol=1e-12, rtol=0)
    cols = catalog_json()["cf_columns"]
    cpos = {s: i for i, s in enumerate(cols)}
    k2 = 2 * int(g3["k"])
    for i, u in enumerate(g3["query_users"]):
        recs = cf.get_recommendations(int(u), k2)
        L = int(g3["lens"][i])
        _eq_lists([cpos[r.set_num] for r in recs], [r.score for r in recs], g3["ids"][i][:L], g3["scores"][i][:L])
        assert all(r.reasons == ["Users with similar preferences also liked this set"] for r in recs)
    # unknown user -> cold start (empty: the synthetic ratings are not in the database)
    assert len(cf.get_recommendations(10 ** 6, 10)) == int(g3["cold_start_len"])


def check_constraint_masks(hy, golden):
    from brickrec.constraints import create_constraint_set_values
    g4 = golden("g4_hybrid.npz")
    rows = catalog_json()["row_set_nums"]
    for ci, cj in enumerate(g4["case_json"]):
        kw = json.loads(str(cj))
        res = hy.constraint_filter.apply_constraints(create_constraint_set_values(**kw))
        want = [s for s, m in zip(rows, g4["masks"][ci]) if m]
        assert res.valid_set_nums == want, f"case {ci} {kw}: {len(res.valid_set_nums)} vs {len(want)}"


def check_hybrid(hy, golden):
    from brickrec.constraints import create_constraint_set_values
    g4 = golden("g4_hybrid.npz")
    rows = catalog_json()["row_set_nums"]
    pos = {s: i for i, s in enumerate(rows)}
    cases = [json.loads(str(c)) for c in g4["case_json"]]
    k = int(g4["k"])
    for case, (u, qrow, ci) in enumerate(g4["hybrid_meta"]):
        cons = create_constraint_set_values(**cases[ci]) if ci >= 0 else None
        recs, res = hy.get_recommendations(user_id=int(u) if u >= 0 else None,
                                           liked_set=rows[int(qrow)] if qrow >= 0 else None,
                                           top_k=k, constraints=cons)
        L = int(g4["lens"][case])
        _eq_lists([pos[r.set_num] for r in recs], [r.score for r in recs], g4["ids"][case][:L],
                  g4["scores"][case][:L])
        if u >= 0 and qrow >= 0:
            # the one-pass device HYBRID path must build the same records as the per-side
            # lists + _combine_recommendations (recommendation_system.py:789-843)
            cf = hy.collaborative_recommender
            m = hy._mask_for(res.valid_mask) if res is not None else None
            c = hy.content_recommender.similar_by_mask(rows[int(qrow)], 2 * k, m)
            f = cf.recommend_by_mask(cf._lookup(int(u)), 2 * k, m)
            if c and f:
                want = hy._combine_recommendations(c, f, k)
                assert [r.set_num for r in recs] == [r.set_num for r in want]
                assert [r.reasons for r in recs] == [r.reasons for r in want]
                assert [(r.name, r.year, r.num_parts, r.theme_name) for r in recs] == \
                    [(r.name, r.year, r.num_parts, r.theme_name) for r in want]
                np.testing.assert_allclose([r.score for r in recs], [r.score for r in want], atol=1e-6)
