"""Semantic (embedding) search drop-in: the PGVector / FAISS retriever of ``NLPRecommender``
(lego_nlp_recommeder.py:288-305, 1379-1412) as an exact cosine scan on the device.

The reference works like this:

1. It encodes the query with MiniLM-L6-v2 (``normalize_embeddings=True``, :143-149).
2. Its retriever returns the k=20 nearest documents by pgvector cosine distance (:305).
3. ``_apply_filters`` drops documents on metadata (:1514-1549).
4. It returns ``[:top_k]`` as dicts whose ``score`` is always 0.0 (:1409).

``SemanticIndex`` keeps the embedding matrix resident in HBM and runs step 2 as one
``bb_search`` in SEMANTIC mode, for one query or a whole batch. Steps 3-4 stay host code,
unchanged.

``search_recommendations`` is the drop-in for ``HuggingFaceNLPRecommender.search_recommendations``
(hf_nlp_recommender.py:1207-1259).  The reference encodes the semantic query and then ignores
the embedding (``_query_vector_database`` runs ``ORDER BY RANDOM()``, :1310-1349); here the
embedding drives an exact cosine KNN over the same candidate rows (num_parts > 50, year >=
2005) — new, documented behaviour — and ``relevance_score`` is the cosine instead of the
constant 0.8.  The theme branch (:1226-1237, ``_query_by_themes`` :1261-1305) and
``_apply_filters`` (:1351-1386) are restated as host code over the metadata.

The query encoder is out of scope: its weights are fetched by name and there is no network
here. Callers pass query vectors, or an ``encoder`` callable that produces them.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

RETRIEVER_K = 20   # lego_nlp_recommeder.py:305  search_kwargs={"k": 20}


def read_faiss_flat(path: str) -> np.ndarray:
    """Vectors of a FAISS ``IndexFlat`` file (``IxF2`` / ``IxFI``): the header, then ntotal·d
    float32 values (e.g. the reference's test_embeddings/index.faiss).

    The file is parsed as data. Nothing in it is executed."""
    b = open(path, "rb").read()
    if b[:4] not in (b"IxF2", b"IxFI"):
        raise ValueError(f"{path}: not a FAISS flat index")
    d = int(np.frombuffer(b, np.int32, 1, 4)[0])
    ntotal = int(np.frombuffer(b, np.int64, 1, 8)[0])
    off = len(b) - ntotal * d * 4
    if off < 16:
        raise ValueError(f"{path}: truncated")
    return np.frombuffer(b, np.float32, ntotal * d, off).reshape(ntotal, d).copy()


def apply_filters(docs: Sequence[Dict], filters: Optional[Dict]) -> List[Dict]:
    """``_apply_filters`` (lego_nlp_recommeder.py:1514-1549) over metadata dicts."""
    if not filters:
        return list(docs)
    out = []
    for m in docs:
        if filters.get("min_pieces") and m["num_parts"] < filters["min_pieces"]:
            continue
        if filters.get("max_pieces") and m["num_parts"] > filters["max_pieces"]:
            continue
        if filters.get("themes"):
            theme = (m.get("theme") or "").lower()
            if not any(t.lower() in theme for t in filters["themes"]):
                continue
        if filters.get("complexity") and m.get("complexity") != filters["complexity"]:
            continue
        if filters.get("min_age") and m["year"] < 2010:
            continue
        out.append(m)
    return out


def hf_apply_filters(results: Sequence[Dict], filters: Optional[Dict]) -> List[Dict]:
    """``HuggingFaceNLPRecommender._apply_filters`` (hf_nlp_recommender.py:1351-1386): exact
    theme-name membership, piece bounds, age bounds when the row carries them."""
    if not filters:
        return list(results)
    out = []
    for r in results:
        if filters.get("themes") and r.get("theme") and r["theme"] not in filters["themes"]:
            continue
        if filters.get("min_pieces") and r.get("num_parts") and r["num_parts"] < filters["min_pieces"]:
            continue
        if filters.get("max_pieces") and r.get("num_parts") and r["num_parts"] > filters["max_pieces"]:
            continue
        if filters.get("min_age") and r.get("min_age") and r["min_age"] > filters["min_age"]:
            continue
        if filters.get("max_age") and r.get("max_age") and r["max_age"] < filters["max_age"]:
            continue
        out.append(r)
    return out


class SemanticIndex:
    """Embedding rows (unit-norm fp32, e.g. MiniLM 384-d) + per-row metadata, on the device."""

    def __init__(self, set_nums: Sequence[str], embeddings: np.ndarray, metadata: Optional[Sequence[Dict]] = None,
                 device: int = 0, dtype: str = "f32", index_factory=None):
        self.set_nums = list(set_nums)
        self.pos = {s: i for i, s in enumerate(self.set_nums)}
        emb = np.asarray(embeddings)
        if emb.shape[0] != len(self.set_nums):
            raise ValueError("one embedding row per set_num")
        self.metadata = list(metadata) if metadata is not None else [{"set_num": s} for s in self.set_nums]
        if index_factory is None:
            from .engine import ItemIndex
            self.index = ItemIndex(device=device, dtype=dtype)
        else:
            self.index = index_factory()
        self.index.upload_items(emb)
        self.d = emb.shape[1]

    @classmethod
    def from_faiss(cls, path: str, set_nums: Sequence[str], metadata=None, **kw) -> "SemanticIndex":
        return cls(set_nums, read_faiss_flat(path), metadata, **kw)

    # ---------------------------------------------------------------- device calls
    def search_vectors(self, queries, k: int, mask: Optional[np.ndarray] = None):
        """Exact cosine top-k for a batch of query vectors (numpy host or torch device).
        Returns (scores [B][k] f32, row ids [B][k] int64 with -1 = empty, counts [B])."""
        q = queries if not isinstance(queries, (list, tuple)) else np.asarray(queries, np.float32)
        if isinstance(q, np.ndarray) and q.ndim == 1:
            q = q[None, :]
        return self.index.search("semantic", k, q_rows=q, mask=mask)

    def similar_to(self, set_nums: Sequence[str], k: int, mask: Optional[np.ndarray] = None):
        """Similar sets of stored rows (rank 0 = the arg-max dropped, as get_similar_sets)."""
        rows = np.array([self.pos[s] for s in set_nums], np.int64)
        return self.index.search("similar", k, q_items=rows, mask=mask)

    # ---------------------------------------------------------------- reference surface
    def semantic_search(self, query, top_k: int = 10, filters: Optional[Dict] = None,
                        encoder: Optional[Callable[[str], np.ndarray]] = None) -> List[Dict]:
        """``NLPRecommender.semantic_search`` (:1379-1412): retriever k=20 -> filters -> [:top_k]."""
        if isinstance(query, str):
            if encoder is None:
                raise RuntimeError("semantic_search on text needs an encoder (the MiniLM query encoder "
                                   "is not bundled); pass encoder= or a query vector")
            query = encoder(query)
        sc, ids, cnt = self.search_vectors(np.asarray(query, np.float32), RETRIEVER_K)
        docs = [self.metadata[int(i)] for i in ids[0][: int(cnt[0])]]
        out = []
        for m in apply_filters(docs, filters)[:top_k]:
            out.append({"set_num": m["set_num"], "name": m.get("name"), "year": m.get("year"),
                        "num_parts": m.get("num_parts"), "theme": m.get("theme"),
                        "description": m.get("description", ""), "score": m.get("score", 0.0)})
        return out

    def _hf_row(self, i: int, relevance: float) -> Dict:
        m = self.metadata[i]
        return {"set_num": m["set_num"], "name": m.get("name"), "year": m.get("year"),
                "num_parts": m.get("num_parts"), "theme": m.get("theme") or "Generic",
                "theme_id": m.get("theme_id"), "img_url": m.get("img_url"), "relevance_score": relevance}

    def search_recommendations(self, processed_query: Dict, top_k: int = 10,
                               encoder: Optional[Callable[[str], np.ndarray]] = None) -> List[Dict]:
        """``HuggingFaceNLPRecommender.search_recommendations`` (hf_nlp_recommender.py:1207-1259).

        ``processed_query`` is the reference's ``process_natural_language_query`` result
        (``semantic_query``, ``filters``, ``confidence``, ``intent``), optionally with a
        precomputed ``embedding``.  Errors return ``[]`` as the reference does (:1257-1259);
        so does a text query with no encoder (the reference's "embedding model not
        available" branch, :1219-1221)."""
        try:
            filters = processed_query.get("filters", {}) or {}
            themes = filters.get("themes", [])
            if themes:  # _query_by_themes (:1261-1305): LIKE %theme%, parts > 50, year >= 2000
                pats = [t.lower() for t in themes]
                rows = [i for i, m in enumerate(self.metadata)
                        if (m.get("num_parts") or 0) > 50 and (m.get("year") or 0) >= 2000
                        and any(p in (m.get("theme") or "").lower() for p in pats)]
                rows.sort(key=lambda i: (-(self.metadata[i].get("num_parts") or 0), -(self.metadata[i].get("year") or 0)))
                results = [self._hf_row(i, 0.9) for i in rows[: top_k * 2]]
                if results:
                    out = hf_apply_filters(results, filters)
                    for r in out:
                        r["confidence"] = processed_query["confidence"]
                        r["intent"] = processed_query["intent"]
                        r["relevance_score"] = 0.9
                    return out[:top_k]
            q = processed_query.get("embedding")
            if q is None:
                if encoder is None:
                    return []
                q = encoder(processed_query["semantic_query"])
            # _query_vector_database's candidate rows (:1316-1327), ranked by cosine
            ok = np.array([(m.get("num_parts") or 0) > 50 and (m.get("year") or 0) >= 2005 for m in self.metadata])
            sc, ids, cnt = self.search_vectors(np.asarray(q, np.float32), top_k, mask=ok)
            results = [self._hf_row(int(i), float(v)) for i, v in zip(ids[0][: int(cnt[0])], sc[0][: int(cnt[0])])]
            out = hf_apply_filters(results, filters)
            for r in out:
                r["confidence"] = processed_query["confidence"]
                r["intent"] = processed_query["intent"]
            return out[:top_k]
        except Exception:
            return []
