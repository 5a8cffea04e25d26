"""Semantic (embedding) search drop-in: the reference's real MiniLM vectors (G5) through
SemanticIndex, the retriever-k=20 + _apply_filters + [:top_k] flow, and the FAISS flat
reader — on CPU with the oracle-backed stand-in (tests/test_gpu_parity.py covers the
same vectors on the device)."""
import numpy as np
import pytest

from _oracle_index import OracleIndex


def _index(golden):
    from brickrec.semantic import SemanticIndex
    g = golden("g5_faiss.npz")
    names = [str(s) for s in g["set_nums"]]
    meta = [{"set_num": s, "name": f"Set {s}", "year": 2000 + i, "num_parts": 100 * (i + 1),
             "theme": "Star Wars" if i % 2 else "Icons", "complexity": "moderate"} for i, s in enumerate(names)]
    return SemanticIndex(names, g["vectors"], meta, index_factory=OracleIndex), g, names


def test_similar_to_known_answer(golden):
    idx, g, names = _index(golden)
    sc, ids, cnt = idx.similar_to(["75192-1"], 3)
    assert [names[int(i)] for i in ids[0]] == ["75331-1", "75313-1", "10294-1"]
    assert abs(sc[0][0] - 0.845918) < 1e-5
    sc, ids, cnt = idx.similar_to(names, len(names) - 1)
    for i in range(len(names)):
        assert list(ids[i]) == list(g["ids"][i])


def test_semantic_search_flow(golden):
    idx, g, names = _index(golden)
    q = g["vectors"][names.index("75192-1")]
    res = idx.semantic_search(q, top_k=3)
    assert [r["set_num"] for r in res][:1] == ["75192-1"]       # its own vector ranks first
    assert all(r["score"] == 0.0 for r in res)                   # as the reference (:1409)
    res = idx.semantic_search(q, top_k=10, filters={"themes": ["star"], "max_pieces": 800})
    assert all("Star" in r["theme"] and r["num_parts"] <= 800 for r in res)
    with pytest.raises(RuntimeError):
        idx.semantic_search("a castle", top_k=3)
    res = idx.semantic_search("a castle", top_k=2, encoder=lambda s: q)
    assert res[0]["set_num"] == "75192-1"


def test_read_faiss_flat(tmp_path, golden):
    from brickrec.semantic import read_faiss_flat
    g = golden("g5_faiss.npz")
    x = g["vectors"]
    hdr = bytearray(int(g["header_offset"]))
    hdr[:4] = b"IxF2"
    hdr[4:8] = np.int32(x.shape[1]).tobytes()
    hdr[8:16] = np.int64(x.shape[0]).tobytes()
    p = tmp_path / "index.faiss"
    p.write_bytes(bytes(hdr) + x.astype(np.float32).tobytes())
    np.testing.assert_array_equal(read_faiss_flat(str(p)), x)
    (tmp_path / "bad").write_bytes(b"nope" + bytes(40))
    with pytest.raises(ValueError):
        read_faiss_flat(str(tmp_path / "bad"))


def test_hf_search_recommendations(golden):
    """HuggingFaceNLPRecommender.search_recommendations drop-in: theme branch (LIKE, parts >
    50, year >= 2000, parts desc), the KNN branch over the reference's candidate rows
    (parts > 50, year >= 2005), _apply_filters, confidence/intent, [] without an encoder."""
    from brickrec.semantic import hf_apply_filters
    idx, g, names = _index(golden)
    pq = {"semantic_query": "star wars ship", "filters": {"themes": ["Star Wars"]}, "confidence": 0.7,
          "intent": "search"}
    res = idx.search_recommendations(pq, top_k=3)
    assert len(res) == 3 and all(r["theme"] == "Star Wars" and r["relevance_score"] == 0.9 for r in res)
    assert [r["num_parts"] for r in res] == sorted((r["num_parts"] for r in res), reverse=True)
    assert all(r["confidence"] == 0.7 and r["intent"] == "search" for r in res)
    q = g["vectors"][names.index("75192-1")]
    pq = {"semantic_query": "x", "filters": {}, "confidence": 0.5, "intent": "search"}
    assert idx.search_recommendations(pq, top_k=3) == []          # no encoder: as the reference
    res = idx.search_recommendations(dict(pq, embedding=q), top_k=3)
    meta = {m["set_num"]: m for m in idx.metadata}
    eligible = [s for s in names if meta[s]["num_parts"] > 50 and meta[s]["year"] >= 2005]
    sims = {s: float(np.dot(q, g["vectors"][names.index(s)])) for s in eligible}
    want = sorted(eligible, key=lambda s: -sims[s])[:3]
    assert [r["set_num"] for r in res] == want
    assert all(abs(r["relevance_score"] - sims[r["set_num"]]) < 1e-5 for r in res)
    res2 = idx.search_recommendations(pq, top_k=3, encoder=lambda s: q)
    assert [r["set_num"] for r in res2] == want
    assert hf_apply_filters([{"theme": "Icons", "num_parts": 10}], {"themes": ["Star Wars"]}) == []
    assert idx.search_recommendations({"filters": None}, top_k=3) == []  # malformed -> []
