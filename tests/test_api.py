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


@pytest.fixture(scope="module")
def client():
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
        app = create_app(conn, index_factory=OracleIndex)
    finally:
        RS._current_year = old
    with TestClient(app) as c:
        yield c


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
