"""CPU restatement of the reference's scoring path — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker / the timed
CPU baseline.  The product path (``brickbrain-rec-engine_amd/brickrec``) never imports it
and has no CPU fallback: it fails loudly when the HIP library is missing.

Parity pinning: every function below is checked in ``tests/test_oracle_golden.py``
against ``tests/golden/*.npz``, which ``oracle/gen_golden.py`` produced by importing and
running the reference's own ``src/scripts/recommendation_system.py`` and
``src/scripts/hard_constraint_filter.py`` (sqlite-backed, psycopg2 stubbed) in the build
container, plus the reference's real MiniLM vectors in ``test_embeddings/index.faiss``.

Tie rule.  The reference orders with an unstable ``np.argsort`` (content path) and a
hash-seeded ``set`` (hybrid union), so its tie order is unspecified
(SURVEY.md §8a rule v).  The restatement fixes it as (score desc, item index asc), which is
what Python's stable ``list.sort(reverse=True)`` gives on the CF path
(recommendation_system.py:460) and what the HIP kernels implement.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np


# ----------------------------------------------------------------------------------------
# cosine similarity with sklearn semantics
# ----------------------------------------------------------------------------------------
def normalize_rows(x: np.ndarray) -> np.ndarray:
    """Row L2 normalisation exactly as ``sklearn.preprocessing.normalize`` does it.

    ``sklearn.metrics.pairwise.cosine_similarity`` (called at
    recommendation_system.py:214) normalises BOTH arguments on every call: norms from
    ``einsum('ij,ij->i')`` in the input dtype, zero norms replaced by 1 (so zero rows
    stay zero and score 0), then a true division.
    """
    x = np.asarray(x)
    norms = np.sqrt(np.einsum("ij,ij->i", x, x))
    norms[norms == 0.0] = 1.0
    return x / norms[:, None]


def cosine_scores(q: np.ndarray, x: np.ndarray) -> np.ndarray:
    """``cosine_similarity(q, x)``: dtype follows the inputs (f32 in -> f32 out)."""
    return normalize_rows(q) @ normalize_rows(x).T


# ----------------------------------------------------------------------------------------
# top-k with the fixed tie rule
# ----------------------------------------------------------------------------------------
def topk_indices(scores: np.ndarray, k: int, allowed: Optional[np.ndarray] = None
                 ) -> Tuple[np.ndarray, np.ndarray]:
    """Top-k of one score row by (score desc, index asc) over ``allowed`` items.

    Returns (indices int64, scores) of length min(k, #allowed).
    """
    scores = np.asarray(scores)
    idx = np.arange(scores.shape[0], dtype=np.int64)
    if allowed is not None:
        idx = idx[np.asarray(allowed, dtype=bool)]
    if k <= 0 or idx.size == 0:
        return idx[:0], scores[:0]
    s = scores[idx]
    if idx.size > 4 * k:
        # keep everything tied with the k-th best, then order exactly
        kth = np.partition(s, idx.size - k)[idx.size - k]
        keep = s >= kth
        idx, s = idx[keep], s[keep]
    order = np.lexsort((idx, -s))[:k]
    return idx[order], s[order]


def rank0(scores: np.ndarray) -> int:
    """Index dropped by ``np.argsort(sim)[::-1][1:]`` (recommendation_system.py:217):
    the arg-max of the UNMASKED row; ties resolved by the fixed rule (lowest index)."""
    s = np.asarray(scores)
    m = s.max()
    return int(np.flatnonzero(s == m)[0])


def similar_sets(x: np.ndarray, query_row: int, k: int,
                 allowed: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
    """``ContentBasedRecommender.get_similar_sets`` (recommendation_system.py:194-249).

    sim = cosine(x[q], x) (:213-214); order = argsort desc, drop rank 0 (:217) — the
    arg-max, not necessarily the query row; walk the order skipping items outside the
    valid filter (:229) until k are accepted.  An empty filter list means "no filter"
    (``if valid_set_filter and ...``), which callers express as ``allowed=None``.
    """
    sim = cosine_scores(x[query_row:query_row + 1], x)[0]
    drop = rank0(sim)
    ok = np.ones(sim.shape[0], dtype=bool) if allowed is None else np.asarray(allowed, bool).copy()
    ok[drop] = False
    return topk_indices(sim, k, ok)


def semantic_topk(x: np.ndarray, q: np.ndarray, k: int,
                  allowed: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Exact cosine KNN of each query row: the sequential scan that pgvector ``<=>``
    (lego_nlp_recommeder.py:296-305, 1394) and FAISS ``IndexFlat`` perform, ranked by
    cosine desc (= cosine distance asc)."""
    sim = cosine_scores(np.atleast_2d(q), x)
    out_i, out_s = [], []
    for row in sim:
        i, s = topk_indices(row, k, allowed)
        out_i.append(i)
        out_s.append(s)
    return out_i, out_s


def cf_topk(user_vec: np.ndarray, item_factors: np.ndarray, k: int,
            allowed: Optional[np.ndarray] = None, rated: Optional[np.ndarray] = None,
            present: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
    """``CollaborativeFilteringRecommender.get_recommendations`` (:411-483).

    scores = u · Fᵀ (:438, no normalisation); skip items the user rated (:441-451) and
    items outside the valid filter (:454); stable sort desc (:460) -> (score desc,
    index asc); top k.  ``present`` marks items that exist in the CF item space (the
    pivot-table columns, :325-336) when ``item_factors`` is laid out in a wider space.
    """
    scores = np.asarray(item_factors) @ np.asarray(user_vec)
    ok = np.ones(scores.shape[0], dtype=bool)
    if allowed is not None:
        ok &= np.asarray(allowed, bool)
    if rated is not None:
        ok &= ~np.asarray(rated, bool)
    if present is not None:
        ok &= np.asarray(present, bool)
    return topk_indices(scores, k, ok)


def union_blend(c_ids: Sequence[int], c_scores: Sequence[float],
                f_ids: Sequence[int], f_scores: Sequence[float],
                w_content: float, w_cf: float, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """``HybridRecommender._combine_recommendations`` (:789-843).

    Over the UNION of both lists: h = wc·c + wcf·cf with a missing side scored 0
    (:812-818); sort desc (:842) -> top k.  Blend in float64 as the reference does.
    """
    cd = {int(i): float(s) for i, s in zip(c_ids, c_scores)}
    fd = {int(i): float(s) for i, s in zip(f_ids, f_scores)}
    ids = sorted(set(cd) | set(fd))
    h = [w_content * cd.get(i, 0.0) + w_cf * fd.get(i, 0.0) for i in ids]
    order = sorted(range(len(ids)), key=lambda j: (-h[j], ids[j]))[:k]
    return (np.array([ids[j] for j in order], dtype=np.int64),
            np.array([h[j] for j in order], dtype=np.float64))


def hybrid(x: np.ndarray, liked_row: Optional[int], user_vec: Optional[np.ndarray],
           item_factors: Optional[np.ndarray], k: int, allowed: Optional[np.ndarray] = None,
           rated: Optional[np.ndarray] = None, present: Optional[np.ndarray] = None,
           w_content: float = 0.4, w_cf: float = 0.6):
    """``HybridRecommender.get_recommendations`` (:612-677), scoring part.

    Each side returns its top 2k (:648-656); one side empty -> the other's top k
    (:659-662); both present -> union blend (:668).  Returns None when neither side
    has results (the reference then runs the popular-sets SQL, :663-665, out of scope).
    """
    c_i = c_s = f_i = f_s = np.zeros(0)
    if liked_row is not None:
        c_i, c_s = similar_sets(x, liked_row, 2 * k, allowed)
    if user_vec is not None:
        f_i, f_s = cf_topk(user_vec, item_factors, 2 * k, allowed, rated, present)
    if len(c_i) == 0 and len(f_i) > 0:
        return f_i[:k], f_s[:k]
    if len(c_i) > 0 and len(f_i) == 0:
        return c_i[:k], c_s[:k]
    if len(c_i) == 0 and len(f_i) == 0:
        return None
    return union_blend(c_i, c_s, f_i, f_s, w_content, w_cf, k)


# ----------------------------------------------------------------------------------------
# hard-constraint mask (hard_constraint_filter.py:318-480)
# ----------------------------------------------------------------------------------------
@dataclass
class Catalog:
    """Item attribute columns in item-index order (the columns the constraint SQL reads)."""
    num_parts: np.ndarray              # int, <=0 or missing -> excluded by "num_parts > 0"
    year: np.ndarray                   # int
    theme_id: np.ndarray               # int, -1 = SQL NULL
    theme_names: Dict[int, str] = field(default_factory=dict)
    owned: Dict[int, set] = field(default_factory=dict)       # user -> item indices
    wishlisted: Dict[int, set] = field(default_factory=dict)  # user -> item indices


def _like_to_regex(pattern: str) -> "re.Pattern":
    """SQL ``LIKE`` -> regex: ``%`` any run, ``_`` one char, everything else literal."""
    out = []
    for ch in pattern:
        out.append(".*" if ch == "%" else "." if ch == "_" else re.escape(ch))
    return re.compile("".join(out), re.DOTALL)


def theme_ids_like(theme_names: Dict[int, str], names: Iterable[str]) -> List[int]:
    """``_get_theme_ids`` (:482-532): ``LOWER(name) LIKE LOWER('%' || n || '%')``, OR-ed."""
    pats = [_like_to_regex(f"%{n}%".lower()) for n in names]
    return sorted(tid for tid, tn in theme_names.items()
                  if any(p.fullmatch(tn.lower()) for p in pats))


def constraint_mask(cat: Catalog, constraints: Sequence[Tuple[str, object]],
                    current_year: int) -> np.ndarray:
    """Mask of items passing every constraint, ANDed with ``num_parts > 0`` (:343).

    ``constraints`` is a list of (constraint_type value string, value) pairs, e.g.
    ("pieces_max", 800).  Predicate map follows ``_constraint_to_sql`` (:366-480),
    including SQL NULL semantics for a missing theme_id (both the ``= ANY`` test and
    its negation are NULL, i.e. the row is dropped).
    """
    parts = np.asarray(cat.num_parts, dtype=np.int64)
    year = np.asarray(cat.year, dtype=np.int64)
    theme = np.asarray(cat.theme_id, dtype=np.int64)
    m = parts > 0
    for ctype, value in constraints:
        if ctype == "pieces_max":
            m &= parts <= value
        elif ctype == "pieces_min":
            m &= parts >= value
        elif ctype == "year_min":
            m &= year >= value
        elif ctype == "year_max":
            m &= year <= value
        elif ctype == "price_max":
            m &= parts <= int(value / 0.10)          # :391-395
        elif ctype == "price_min":
            m &= parts >= int(value / 0.15)          # :397-400
        elif ctype == "themes_required":             # :402-409
            ids = theme_ids_like(cat.theme_names, value)
            m &= np.isin(theme, ids) & (theme >= 0) if ids else np.zeros_like(m)
        elif ctype == "themes_excluded":             # :411-418
            ids = theme_ids_like(cat.theme_names, value)
            if ids:
                m &= ~np.isin(theme, ids) & (theme >= 0)
        elif ctype == "age_min":                     # :420-430
            if value <= 4:
                m &= parts <= 50
            elif value <= 8:
                m &= parts <= 500
            elif value <= 12:
                m &= parts <= 1500
            else:
                m &= parts >= 500
        elif ctype == "age_max":                     # :432-439
            if value <= 8:
                m &= parts <= 300
            elif value <= 12:
                m &= parts <= 800
        elif ctype == "exclude_owned":               # :441-445
            own = cat.owned.get(value, set())
            if own:
                m[list(own)] = False
        elif ctype == "exclude_wishlisted":          # :447-451
            wl = cat.wishlisted.get(value, set())
            if wl:
                m[list(wl)] = False
        elif ctype == "complexity_max":              # :453-461
            m &= parts <= {"simple": 200, "moderate": 800, "complex": 999999}.get(value, 999999)
        elif ctype == "complexity_min":              # :463-471
            m &= parts >= {"simple": 0, "moderate": 200, "complex": 800}.get(value, 0)
        elif ctype == "availability":                # :473-477
            m &= year >= current_year - 5
    return m


def unit_rows(n: int, d: int, seed: int) -> np.ndarray:
    """Synthetic unit-norm fp32 rows (N(0,1) rows, L2-normalised)."""
    x = np.random.default_rng(seed).standard_normal((n, d)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x


# ----------------------------------------------------------------------------------------
# bench helper: bounded CPU baseline of the same workload
# ----------------------------------------------------------------------------------------
def batched_cosine_topk(x_normed: np.ndarray, q: np.ndarray, k: int
                        ) -> Tuple[np.ndarray, np.ndarray]:
    """Batched exact cosine top-k with the items already normalised once (what a
    sequential-scan index holds); queries normalised per call as sklearn does."""
    sim = normalize_rows(q) @ x_normed.T
    n = sim.shape[1]
    part = np.argpartition(-sim, k - 1, axis=1)[:, :k]
    ps = np.take_along_axis(sim, part, axis=1)
    order = np.lexsort((part, -ps), axis=1)
    return (np.take_along_axis(part, order, axis=1).astype(np.int64),
            np.take_along_axis(ps, order, axis=1))
