"""FastAPI drop-in routes (brickrec.api) over the reference's synthetic catalogue, on CPU with
the oracle-backed index stand-in: request/response fields and orderings against the
reference's golden outputs (G1 content, G3 CF, G4 hybrid + constraints)."""
import json
import sqlite3

import numpy as np
import pytest

import _dropin_checks as D
from _oracle_index import OracleIndex
from _spaces import catalog_json


def make_client(index_factory):
    """The app over the golden catalogue with the given index (OracleIndex on CPU, None = the
    HIP ItemIndex); yields a TestClient."""
    pytest.importorskip("httpx")
    from fastapi.testclient import TestClient
    from oracle.gen_golden import PgOnSqlite
    import brickrec.recommenders as RS
    from brickrec.api import create_app
    world = D.build_world()
    # the app serves from worker threads: hand it a thread-shareable copy of the database
    db = sqlite3.connect(":memory:", check_same_thread=False)
    world._db.backup(db)
    conn = PgOnSqlite(db, D._DictRows)
    year = int(catalog_json()["generated_year"])
    old = RS._current_year
    RS._current_year = lambda: year
    try:
        app = create_app(conn, index_factory=index_factory)
    finally:
        RS._current_year = old
    with TestClient(app) as c:
        yield c


@pytest.fixture(scope="module")
def client():
    yield from make_client(OracleIndex)


def test_health(client):
    r = client.get("/health")
    assert r.status_code == 200 and r.json()["status"] == "healthy"


def test_content_route_matches_reference(client, golden):
    g1 = golden("g1_content.npz")
    cat = catalog_json()
    rows = cat["row_set_nums"]
    q = int(g1["query_rows"][0])
    r = client.post("/recommendations", json={"set_num": rows[q], "top_k": 50, "recommendation_type": "content"})
    assert r.status_code == 200, r.text
    body = r.json()
    assert [rows.index(x["set_num"]) for x in body] == list(g1["ids_nofilter"][0])
    np.testing.assert_allclose([x["score"] for x in body], g1["scores_nofilter"][0], atol=1e-5)
    assert [x["reasons"] for x in body] == cat["g1_reasons_nofilter"][0]
    assert set(body[0]) == {"set_num", "name", "score", "reasons", "theme_name", "year", "num_parts", "img_url",
                            "constraint_violations"}
    r = client.post("/recommendations", json={"set_num": rows[q], "top_k": 5, "recommendation_type": "content",
                                              "include_reasons": False})
    assert all(x["reasons"] == [] for x in r.json())


def test_collaborative_route(client, golden):
    g3 = golden("g3_cf.npz")
    cols = catalog_json()["cf_columns"]
    r = client.post("/recommendations", json={"user_id": int(g3["query_users"][0]), "top_k": 20,
                                              "recommendation_type": "collaborative"})
    assert r.status_code == 200, r.text
    L = int(g3["lens"][0])
    assert [cols.index(x["set_num"]) for x in r.json()] == list(g3["ids"][0][:L])


def test_hybrid_route_returns_list(client, golden):
    g4 = golden("g4_hybrid.npz")
    rows = catalog_json()["row_set_nums"]
    case = [i for i, m in enumerate(g4["hybrid_meta"]) if m[2] < 0 and m[0] >= 0 and m[1] >= 0][0]
    u, qrow, _ = g4["hybrid_meta"][case]
    r = client.post("/recommendations", json={"user_id": int(u), "set_num": rows[int(qrow)], "top_k": int(g4["k"])})
    assert r.status_code == 200, r.text
    L = int(g4["lens"][case])
    assert [rows.index(x["set_num"]) for x in r.json()] == list(g4["ids"][case][:L])


def test_constrained_route(client, golden):
    g4 = golden("g4_hybrid.npz")
    rows = catalog_json()["row_set_nums"]
    cases = [json.loads(str(c)) for c in g4["case_json"]]
    for case, (u, qrow, ci) in enumerate(g4["hybrid_meta"]):
        if ci < 0:
            continue
        body = dict(cases[ci])
        if u >= 0:
            body["user_id"] = int(u)
        if qrow >= 0:
            body["set_num"] = rows[int(qrow)]
        body["top_k"] = int(g4["k"])
        r = client.post("/recommendations/constrained", json=body)
        assert r.status_code == 200, r.text
        out = r.json()
        L = int(g4["lens"][case])
        assert [rows.index(x["set_num"]) for x in out["recommendations"]] == list(g4["ids"][case][:L])
        assert out["constraint_summary"]["valid_sets_found"] == int(g4["masks"][ci].sum())


def test_similar_semantic_sql_route(client):
    rows = catalog_json()["row_set_nums"]
    r = client.post("/sets/similar/semantic", json={"set_num": rows[10], "top_k": 5, "description": "easier"})
    assert r.status_code == 200, r.text
    res = r.json()
    diffs = [x["relevance_score"] for x in res]
    assert all(0.1 <= d <= 1.0 for d in diffs)
    assert all("Considering: easier" in x["match_reasons"] for x in res)
    assert client.post("/sets/similar/semantic", json={"set_num": "nope-1"}).status_code == 404


def test_similar_semantic_sql_pinned(client, golden):
    """a14 pinned on the golden catalogue, computed here independently of brickrec.api: the
    reference route (recommendation_api.py:1531-1558) returns sets of the target's theme with
    num_parts in [max(1, int(0.5 p)), int(1.5 p)], num_parts > 0, the target excluded,
    ordered by |Δparts| asc then year desc, LIMIT top_k, relevance max(0.1, 1 − Δ/max(p, p')).
    Rows tied on (Δ, year) have no SQL order, so the comparison is per (Δ, year) group."""
    g1 = golden("g1_content.npz")
    cat = catalog_json()
    rows = cat["row_set_nums"]
    parts, year, theme = g1["num_parts"].astype(np.int64), g1["year"].astype(np.int64), g1["theme_id"]
    checked = 0
    for t in range(0, len(rows), 97):
        p = int(parts[t])
        lo, hi = max(1, int(p * 0.5)), int(p * 1.5)
        cand = np.flatnonzero((theme == theme[t]) & (parts > 0) & (parts >= lo) & (parts <= hi)
                              & (np.arange(len(rows)) != t))
        diff = np.abs(parts[cand] - p)
        order = np.lexsort((-year[cand], diff))
        top_k = 10
        exp = cand[order][:top_k]
        r = client.post("/sets/similar/semantic", json={"set_num": rows[t], "top_k": top_k})
        assert r.status_code == 200, r.text
        res = r.json()
        assert len(res) == len(exp)
        got_keys = [(abs(x["num_parts"] - p), -x["year"]) for x in res]
        assert got_keys == [(int(abs(parts[i] - p)), -int(year[i])) for i in exp]
        for x in res:
            i = rows.index(x["set_num"])
            assert theme[i] == theme[t] and lo <= parts[i] <= hi and i != t
            rel = max(0.1, 1.0 - abs(int(parts[i]) - p) / max(p, int(parts[i])))
            assert x["relevance_score"] == pytest.approx(rel, abs=1e-12)
            assert x["match_reasons"][:2] == [f"Same theme: {cat['theme_names'][i]}",
                                              f"Similar size: {int(parts[i])} vs {p} pieces"]
        # tie groups of (Δ, year) hold the same sets in any order
        for key in set(got_keys):
            assert ({x["set_num"] for x, kk in zip(res, got_keys) if kk == key} <=
                    {rows[i] for i in cand if (int(abs(parts[i] - p)), -int(year[i])) == key})
        checked += len(res) > 0
    assert checked >= 5


def test_embedding_route_is_opt_in(client):
    """The embedding KNN is a separate route; without a SemanticIndex it refuses."""
    assert client.post("/sets/similar/embedding", json={"set_num": "x"}).status_code == 400


def test_errors(client):
    assert client.post("/recommendations", json={"recommendation_type": "content"}).status_code == 400
    assert client.post("/recommendations", json={"set_num": "x", "top_k": 0}).status_code == 422
    assert client.post("/recommendations", json={"set_num": "no-such", "recommendation_type": "content"}).json() == []


def test_batch_route(client, golden):
    g1 = golden("g1_content.npz")
    rows = catalog_json()["row_set_nums"]
    qs = [rows[int(q)] for q in g1["query_rows"][:4]]
    r = client.post("/recommendations/batch", json={"set_nums": qs, "top_k": 50})
    assert r.status_code == 200, r.text
    for b, names in enumerate(r.json()["set_nums"]):
        assert [rows.index(s) for s in names] == list(g1["ids_nofilter"][b])
