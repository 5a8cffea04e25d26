"""GPU parity of the semantic drop-ins on the HIP index.

* ``SemanticIndex.semantic_search`` = ``NLPRecommender.semantic_search``
  (lego_nlp_recommeder.py:1379-1412): retriever k=20 (:305), ``_apply_filters``
  (:1514-1549), ``[:top_k]``, score 0.0 (:1409).
* ``SemanticIndex.search_recommendations`` = ``HuggingFaceNLPRecommender.search_recommendations``
  (hf_nlp_recommender.py:1207-1259): theme branch, then the KNN over the reference's
  candidate rows (num_parts > 50, year >= 2005) where the reference draws ORDER BY RANDOM()
  (:1318-1328; documented new behaviour), ``_apply_filters`` (:1351-1386).

The checker restates the flow independently here over the oracle's exact cosine top-k
(oracle/restatement.py semantic_topk): first on the reference's real MiniLM vectors (G5),
then on a 25,216-row synthetic catalogue with metadata, so that the filters bite and the
retriever's 20 rows are a real cut.  pgvector's own arithmetic is parity-unpinned
(SURVEY §8c); the ranking is the sklearn/numpy cosine's.
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


def _filters_ref(docs, filters):
    """_apply_filters (lego_nlp_recommeder.py:1514-1549), restated independently."""
    out = []
    for m in docs:
        f = filters or {}
        if f.get("min_pieces") and m["num_parts"] < f["min_pieces"]:
            continue
        if f.get("max_pieces") and m["num_parts"] > f["max_pieces"]:
            continue
        if f.get("themes") and not any(t.lower() in (m.get("theme") or "").lower() for t in f["themes"]):
            continue
        if f.get("complexity") and m.get("complexity") != f["complexity"]:
            continue
        if f.get("min_age") and m["year"] < 2010:
            continue
        out.append(m)
    return out


def _catalogue(n, seed):
    rng = np.random.default_rng(seed)
    x = R.unit_rows(n, 384, seed)
    themes = ["Star Wars", "Icons", "Technic", "City", "Harry Potter", "Ideas"]
    meta = [{"set_num": f"{10000 + i}-1", "name": f"Set {i}", "year": int(rng.integers(1990, 2025)),
             "num_parts": int(rng.integers(10, 4000)), "theme": themes[int(rng.integers(0, len(themes)))],
             "complexity": ["simple", "moderate", "complex"][int(rng.integers(0, 3))]} for i in range(n)]
    return x, meta


@pytest.mark.parametrize("case", ["g5", "catalogue"])
def test_semantic_search_flow_on_device(brickrec, golden, case):
    from brickrec.semantic import SemanticIndex
    if case == "g5":
        g = golden("g5_faiss.npz")
        x = g["vectors"]
        names = [str(s) for s in g["set_nums"]]
        meta = [{"set_num": s, "name": f"Set {s}", "year": 2000 + i, "num_parts": 100 * (i + 1),
                 "theme": "Star Wars" if i % 2 else "Icons", "complexity": "moderate"} for i, s in enumerate(names)]
        queries = [x[i] for i in range(len(names))]
    else:
        x, meta = _catalogue(25216, 77)
        names = [m["set_num"] for m in meta]
        queries = list(R.unit_rows(24, 384, 78)) + [x[5], x[20000]]
    idx = SemanticIndex(names, x, meta)
    filt = [None, {"themes": ["star"]}, {"max_pieces": 800, "min_age": 8}, {"complexity": "simple"}]
    for q in queries:
        ri, _ = R.semantic_topk(x, q, 20)            # the retriever's k=20, exact cosine
        docs = [meta[int(i)] for i in ri[0]]
        for f in filt:
            for top_k in (3, 10):
                got = idx.semantic_search(np.asarray(q, np.float32), top_k=top_k, filters=f)
                want = _filters_ref(docs, f)[:top_k]
                assert [r["set_num"] for r in got] == [m["set_num"] for m in want]
                assert all(r["score"] == 0.0 for r in got)
    if case == "g5":   # the SURVEY's known answer through the whole flow
        q = x[names.index("75192-1")]
        assert [r["set_num"] for r in idx.semantic_search(q, top_k=4)] == ["75192-1", "75331-1", "75313-1", "10294-1"]


def test_search_recommendations_on_device(brickrec):
    from brickrec.semantic import SemanticIndex
    x, meta = _catalogue(25216, 91)
    names = [m["set_num"] for m in meta]
    idx = SemanticIndex(names, x, meta)
    ok = np.array([m["num_parts"] > 50 and m["year"] >= 2005 for m in meta])
    for j, q in enumerate(R.unit_rows(12, 384, 92)):
        for top_k in (5, 20):
            pq = {"semantic_query": "x", "filters": {"max_pieces": 2000} if j % 2 else {}, "confidence": 0.6,
                  "intent": "search", "embedding": q}
            res = idx.search_recommendations(pq, top_k=top_k)
            ri, rs = R.semantic_topk(x, q, top_k, allowed=ok)      # KNN over the candidate rows
            want = [(names[int(i)], float(s)) for i, s in zip(ri[0], rs[0])
                    if not (j % 2) or meta[int(i)]["num_parts"] <= 2000][:top_k]
            assert [r["set_num"] for r in res] == [w[0] for w in want]
            np.testing.assert_allclose([r["relevance_score"] for r in res], [w[1] for w in want], atol=1e-5)
            assert all(r["confidence"] == 0.6 and r["intent"] == "search" for r in res)
    # theme branch: LIKE %theme%, num_parts > 50, year >= 2000, num_parts desc, relevance 0.9
    res = idx.search_recommendations({"semantic_query": "x", "filters": {"themes": ["Technic"]}, "confidence": 0.5,
                                      "intent": "search"}, top_k=4)
    rows = sorted([m for m in meta if m["num_parts"] > 50 and m["year"] >= 2000 and "technic" in m["theme"].lower()],
                  key=lambda m: (-m["num_parts"], -m["year"]))
    assert [r["set_num"] for r in res] == [m["set_num"] for m in rows[:4]]
