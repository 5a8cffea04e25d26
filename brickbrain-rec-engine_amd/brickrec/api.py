"""FastAPI routes of the hot path — drop-in for the matching routes of
``src/scripts/recommendation_api.py``:

* ``POST /recommendations`` (:432-498);
* ``POST /recommendations/constrained`` (:501-597);
* ``POST /sets/similar/semantic`` (:1501-1585);
* ``GET /health``.

Request and response models carry the reference's field names and validation. One
endpoint is new: ``POST /recommendations/batch`` runs many similar-set / semantic queries
as one device call. The reference's other routes (users, auth, NL parsing, metrics,
conversation) are outside this path.

Behaviour differences, all fixes of reference bugs:

* A hybrid ``/recommendations`` returns the list. The reference iterated the
  (list, result) tuple and always answered 500.
* A collaborative request resolves ``str(user_id)`` to the user. The reference's lookup
  missed it and always fell back to cold start.
* An invalid type / parameter combination is a 400. The reference's own HTTPException was
  caught and re-raised as a 500.

``/sets/similar/semantic`` runs an embedding KNN when the app holds a ``SemanticIndex``.
Without one, it runs the reference's live SQL heuristic: same theme, pieces within ±50 %,
ordered by piece difference.
"""
from __future__ import annotations

import logging
import threading
from typing import Any, Dict, List, Optional, Sequence

from fastapi import FastAPI, HTTPException
from pydantic import BaseModel, Field

from .catalog import Engine, query_rows
from .recommenders import HybridRecommender
from .recommenders import RecommendationRequest as InternalRecommendationRequest

logger = logging.getLogger(__name__)


class RecommendationRequest(BaseModel):
    """recommendation_api.py:240-245"""
    user_id: Optional[int] = None
    set_num: Optional[str] = None
    top_k: int = Field(10, ge=1, le=50)
    recommendation_type: str = Field("hybrid", pattern="^(content|collaborative|hybrid)$")
    include_reasons: bool = True


class EnhancedRecommendationRequest(BaseModel):
    """recommendation_api.py:247-274"""
    user_id: Optional[int] = None
    set_num: Optional[str] = None
    top_k: int = Field(10, ge=1, le=50)
    recommendation_type: str = Field("hybrid", pattern="^(content|collaborative|hybrid)$")
    include_reasons: bool = True
    price_max: Optional[float] = Field(None, ge=0)
    price_min: Optional[float] = Field(None, ge=0)
    pieces_max: Optional[int] = Field(None, ge=1)
    pieces_min: Optional[int] = Field(None, ge=1)
    age_min: Optional[int] = Field(None, ge=1, le=99)
    age_max: Optional[int] = Field(None, ge=1, le=99)
    year_min: Optional[int] = Field(None, ge=1950)
    year_max: Optional[int] = Field(None, le=2030)
    required_themes: Optional[List[str]] = None
    excluded_themes: Optional[List[str]] = None
    max_complexity: Optional[str] = Field(None, pattern="^(simple|moderate|complex)$")
    min_complexity: Optional[str] = Field(None, pattern="^(simple|moderate|complex)$")
    must_be_available: bool = False
    exclude_owned: bool = False
    exclude_wishlisted: bool = False
    preferred_themes: Optional[List[str]] = None
    budget_preference: Optional[float] = Field(None, ge=0)


class RecommendationResponse(BaseModel):
    """recommendation_api.py:276-285"""
    set_num: str
    name: str
    score: float
    reasons: List[str]
    theme_name: Optional[str]
    year: int
    num_parts: int
    img_url: Optional[str]
    constraint_violations: Optional[List[str]] = None


class ConstraintViolationResponse(BaseModel):
    constraint_description: str
    violating_count: int
    total_count: int
    elimination_rate: float
    suggested_alternatives: List[str]


class EnhancedRecommendationResponse(BaseModel):
    recommendations: List[RecommendationResponse]
    constraint_summary: Dict[str, Any]
    violations: List[ConstraintViolationResponse]
    performance_stats: Dict[str, Any]


class SimilarSetQuery(BaseModel):
    """recommendation_api.py:372-375"""
    set_num: str
    description: Optional[str] = None
    top_k: int = Field(10, ge=1, le=50)


class NLSearchResult(BaseModel):
    """recommendation_api.py:354-362"""
    set_num: str
    name: str
    theme: Optional[str]
    year: int
    num_parts: int
    relevance_score: float
    match_reasons: List[str]
    description: str


class BatchQuery(BaseModel):
    """New: many similar-set (set_nums) or semantic (vectors) queries in one device call."""
    set_nums: Optional[List[str]] = None
    vectors: Optional[List[List[float]]] = None
    top_k: int = Field(10, ge=1, le=512)


class BatchResult(BaseModel):
    set_nums: List[List[str]]
    scores: List[List[float]]


def _resp(rec, include_reasons=True, violations=False):
    return RecommendationResponse(set_num=rec.set_num, name=rec.name, score=rec.score,
                                  reasons=rec.reasons if include_reasons else [], theme_name=rec.theme_name,
                                  year=rec.year, num_parts=rec.num_parts, img_url=rec.img_url,
                                  constraint_violations=rec.constraint_violations if violations else None)


def create_app(dbcon, *, engine: Optional[Engine] = None, semantic=None, prepare: bool = True,
               index_factory=None) -> FastAPI:
    """Build the app around one shared engine (the reference's global HybridRecommender,
    recommendation_api.py:44-67).  Calls are serialised by a lock, as the reference's
    single worker + unlocked globals effectively were."""
    eng = engine if engine is not None else Engine(dbcon, index_factory=index_factory)
    rec = HybridRecommender(dbcon, eng)
    if prepare:
        rec.content_recommender.prepare_features()
        rec.collaborative_recommender.prepare_user_item_matrix()
    lock = threading.Lock()
    app = FastAPI(title="brickrec", version="0.1.0")
    app.state.recommender = rec
    app.state.semantic = semantic

    @app.get("/health")
    def health():
        cat = eng.catalog
        return {"status": "healthy", "items": cat.n if cat else 0,
                "content_ready": rec.content_recommender.feat_matrix is not None,
                "cf_ready": rec.collaborative_recommender.svd_model is not None,
                "semantic_ready": semantic is not None}

    @app.post("/recommendations", response_model=List[RecommendationResponse])
    def get_recommendations(request: RecommendationRequest):
        try:
            with lock:
                if request.recommendation_type == "content" and request.set_num:
                    recs = rec.content_recommender.get_similar_sets(request.set_num, request.top_k)
                elif request.recommendation_type == "collaborative" and request.user_id:
                    recs = rec.collaborative_recommender.get_recommendations(str(request.user_id), request.top_k)
                elif request.recommendation_type == "hybrid":
                    recs, _ = rec.get_recommendations(user_id=request.user_id, liked_set=request.set_num,
                                                      top_k=request.top_k)
                else:
                    raise HTTPException(status_code=400,
                                        detail="Invalid recommendation type or missing required parameters")
            return [_resp(r, request.include_reasons) for r in recs]
        except HTTPException:
            raise
        except Exception as e:
            logger.error(f"Error generating recommendations: {e}")
            raise HTTPException(status_code=500, detail=str(e))

    @app.post("/recommendations/constrained", response_model=EnhancedRecommendationResponse)
    def get_constrained_recommendations(request: EnhancedRecommendationRequest):
        try:
            internal = InternalRecommendationRequest(
                user_id=request.user_id, liked_set=request.set_num, top_k=request.top_k,
                price_max=request.price_max, price_min=request.price_min, pieces_max=request.pieces_max,
                pieces_min=request.pieces_min, age_min=request.age_min, age_max=request.age_max,
                year_min=request.year_min, year_max=request.year_max, required_themes=request.required_themes,
                excluded_themes=request.excluded_themes, max_complexity=request.max_complexity,
                min_complexity=request.min_complexity, must_be_available=request.must_be_available,
                exclude_owned=request.exclude_owned, exclude_wishlisted=request.exclude_wishlisted,
                preferred_themes=request.preferred_themes, budget_preference=request.budget_preference)
            with lock:
                recs, cres = rec.get_recommendations_from_request(internal)
            out = [_resp(r, request.include_reasons, violations=True) for r in recs]
            viol = []
            if cres and cres.violations:
                for v in cres.violations:
                    viol.append(ConstraintViolationResponse(
                        constraint_description=v.constraint.description, violating_count=v.violating_count,
                        total_count=v.total_count, elimination_rate=v.violating_count / max(v.total_count, 1),
                        suggested_alternatives=v.suggested_alternatives or []))
            summary = {
                "total_constraints_applied": len(cres.applied_constraints) if cres else 0,
                "valid_sets_found": len(cres.valid_set_nums) if cres else 0,
                "recommendations_returned": len(out),
                "constraint_sql_generated": cres.constraint_sql if cres else "",
                "filtering_effective": len(out) > 0,
            }
            return EnhancedRecommendationResponse(recommendations=out, constraint_summary=summary,
                                                  violations=viol,
                                                  performance_stats=cres.performance_stats if cres else {})
        except HTTPException:
            raise
        except Exception as e:
            logger.error(f"Error generating constrained recommendations: {e}")
            raise HTTPException(status_code=500, detail=str(e))

    @app.post("/sets/similar/semantic", response_model=List[NLSearchResult])
    def similar_semantic(query: SimilarSetQuery):
        """The reference route's live behaviour (recommendation_api.py:1501-1585): the SQL
        theme + piece-count heuristic, whatever index the app holds.  The reference runs it
        on a fresh connection (:1513); here it runs under the app lock on the shared one."""
        try:
            with lock:
                return _similar_by_sql(dbcon, query)
        except HTTPException:
            raise
        except Exception as e:
            logger.error(f"Semantic similarity search error: {e}")
            raise HTTPException(status_code=500, detail=f"Database error: {str(e)}")

    @app.post("/sets/similar/embedding", response_model=List[NLSearchResult])
    def similar_embedding(query: SimilarSetQuery):
        """New route (no reference counterpart): embedding KNN of the stored set over the
        loaded SemanticIndex — the branch the reference route never reaches (:1587-1759)."""
        if semantic is None:
            raise HTTPException(status_code=400, detail="no semantic index loaded")
        try:
            with lock:
                return _similar_by_embedding(semantic, query)
        except HTTPException:
            raise
        except Exception as e:
            logger.error(f"Embedding similarity search error: {e}")
            raise HTTPException(status_code=500, detail=str(e))

    @app.post("/recommendations/batch", response_model=BatchResult)
    def batch(q: BatchQuery):
        import numpy as np
        with lock:
            if q.vectors is not None:
                if semantic is None:
                    raise HTTPException(status_code=400, detail="no semantic index loaded")
                sc, ids, cnt = semantic.search_vectors(np.asarray(q.vectors, np.float32), q.top_k)
                names = semantic.set_nums
            elif q.set_nums is not None:
                cb = rec.content_recommender
                if cb.feat_matrix is None:
                    cb.prepare_features()
                cat = eng.catalog
                missing = [s for s in q.set_nums if s not in cb._row_of_set]
                if missing:
                    raise HTTPException(status_code=404, detail=f"unknown sets: {missing[:5]}")
                rows = np.array([cat.pos[s] for s in q.set_nums], np.int64)
                sc, ids, cnt = eng.ensure_index().search("similar", q.top_k, q_items=rows)
                names = cat.set_nums
            else:
                raise HTTPException(status_code=400, detail="set_nums or vectors required")
        return BatchResult(set_nums=[[names[int(i)] for i in ids[b][: int(cnt[b])]] for b in range(len(cnt))],
                           scores=[[float(s) for s in sc[b][: int(cnt[b])]] for b in range(len(cnt))])

    return app


def _similar_by_sql(dbcon, query: SimilarSetQuery) -> List[NLSearchResult]:
    """The reference's live behaviour of /sets/similar/semantic (:1517-1576)."""
    t = query_rows(dbcon, "SELECT s.*, t.name as theme_name FROM sets s LEFT JOIN themes t ON s.theme_id = t.id "
                          "WHERE s.set_num = %s", [query.set_num])
    if not t:
        raise HTTPException(status_code=404, detail="Set not found")
    t = t[0]
    rows = query_rows(dbcon, """
        SELECT s.set_num, s.name, t.name as theme_name, s.year, s.num_parts,
               ABS(s.num_parts - %s) as piece_diff
        FROM sets s
        LEFT JOIN themes t ON s.theme_id = t.id
        WHERE s.set_num != %s
          AND s.theme_id = %s
          AND s.num_parts > 0
          AND s.num_parts BETWEEN %s AND %s
        ORDER BY piece_diff ASC, s.year DESC
        LIMIT %s""", [t["num_parts"], query.set_num, t["theme_id"], max(1, int(t["num_parts"] * 0.5)),
                      int(t["num_parts"] * 1.5), query.top_k])
    out = []
    for r in rows:
        sim = 1.0 - (r["piece_diff"] / max(t["num_parts"], r["num_parts"]))
        reasons = [f"Same theme: {r['theme_name']}", f"Similar size: {r['num_parts']} vs {t['num_parts']} pieces"]
        if query.description:
            reasons.append(f"Considering: {query.description}")
        out.append(NLSearchResult(set_num=r["set_num"], name=r["name"], theme=r["theme_name"], year=r["year"],
                                  num_parts=r["num_parts"], relevance_score=max(0.1, sim), match_reasons=reasons,
                                  description=f"{r['name']} - {r['num_parts']} pieces from {r['year']}"))
    return out


def _similar_by_embedding(semantic, query: SimilarSetQuery) -> List[NLSearchResult]:
    """Embedding KNN of the stored set (served by the opt-in /sets/similar/embedding route)."""
    if query.set_num not in semantic.pos:
        raise HTTPException(status_code=404, detail="Set not found")
    sc, ids, cnt = semantic.similar_to([query.set_num], query.top_k)
    out = []
    for i, s in zip(ids[0][: int(cnt[0])], sc[0][: int(cnt[0])]):
        m = semantic.metadata[int(i)]
        reasons = ["Semantically similar description"]
        if query.description:
            reasons.append(f"Considering: {query.description}")
        out.append(NLSearchResult(set_num=m["set_num"], name=m.get("name") or m["set_num"], theme=m.get("theme"),
                                  year=int(m.get("year") or 0), num_parts=int(m.get("num_parts") or 0),
                                  relevance_score=float(s), match_reasons=reasons,
                                  description=m.get("description") or ""))
    return out
