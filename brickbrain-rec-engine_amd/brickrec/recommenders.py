"""Drop-ins for ``src/scripts/recommendation_system.py``.

The class names, constructors, method signatures, attributes and return types are the
reference's.  Its scoring loops are replaced by calls into the device index:

* ``ContentBasedRecommender.get_similar_sets`` (:194-249). The reference runs the cosine
  against every row, then argsort, drops rank 0 and walks the filter. Here it is one
  ``bb_search`` in SIMILAR mode.
* ``CollaborativeFilteringRecommender.get_recommendations`` (:411-483). The reference
  computes u·Fᵀ, skips rated and filtered items, and sorts. Here it is one ``bb_search``
  in CF mode, with the rated items as the per-query exclusion bitset.
* ``HybridRecommender``. Each side is one device call; the union blend follows
  ``_combine_recommendations`` (:789-843). ``recommend_batch`` runs the whole hybrid
  (both sides, blend and constraint mask) for many queries in one device call.

Startup work stays host code:

* the ``prepare_features`` feature engineering (pandas / sklearn StandardScaler, as in the
  reference);
* the synthetic ratings and ``TruncatedSVD``.

Those are restated in the reference's exact arithmetic, and tests pin them against the
reference's golden outputs. The only deliberate differences are these:

* Ties order by (score desc, catalogue row asc). The reference's tie order is unspecified:
  it uses an unstable argsort and a hash-seeded set.
* Scores come from the fp32 device path (within 1e-5 of the reference's f64).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from datetime import datetime
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd

from .catalog import Engine
from .constraints import ConstraintResult, HardConstraint, HardConstraintFilter

logger = logging.getLogger(__name__)


def _read_sql(sql, con, params=None):
    """pd.read_sql on a plain DB-API connection (psycopg2, as the reference), without
    pandas' "only SQLAlchemy is tested" warning."""
    import warnings
    with warnings.catch_warnings():
        warnings.filterwarnings("ignore", message="pandas only supports SQLAlchemy")
        return pd.read_sql(sql, con, params=params)


def _current_year() -> int:
    """Clock used by the age score (recommendation_system.py:156); patchable in tests."""
    return datetime.now().year


@dataclass
class RecommendationResult:
    """recommendation_system.py:25-36"""
    set_num: str
    name: str
    score: float
    reasons: List[str]
    theme_name: str
    year: int
    num_parts: int
    img_url: Optional[str] = None
    constraint_violations: Optional[List[str]] = None


@dataclass
class RecommendationRequest:
    """recommendation_system.py:38-63"""
    user_id: Optional[int] = None
    liked_set: Optional[str] = None
    top_k: int = 10
    price_max: Optional[float] = None
    price_min: Optional[float] = None
    pieces_max: Optional[int] = None
    pieces_min: Optional[int] = None
    age_min: Optional[int] = None
    age_max: Optional[int] = None
    year_min: Optional[int] = None
    year_max: Optional[int] = None
    required_themes: Optional[List[str]] = None
    excluded_themes: Optional[List[str]] = None
    max_complexity: Optional[str] = None
    min_complexity: Optional[str] = None
    must_be_available: bool = False
    exclude_owned: bool = False
    exclude_wishlisted: bool = False
    preferred_themes: Optional[List[str]] = None
    preferred_complexity: Optional[str] = None
    budget_preference: Optional[float] = None


_FEATURE_SQL = """
        SELECT
            s.set_num,
            s.name,
            s.year,
            s.theme_id,
            s.num_parts,
            s.img_url,
            t.name as theme_name,
            t.parent_id as parent_theme_id,
            COUNT(DISTINCT ip.part_num) as unique_parts,
            COUNT(DISTINCT ip.color_id) as unique_colors,
            AVG(CASE WHEN ip.is_spare THEN 0 ELSE ip.quantity END) as avg_part_quantity
        FROM sets s
        LEFT JOIN themes t ON s.theme_id = t.id
        LEFT JOIN inventories i ON s.set_num = i.set_num
        LEFT JOIN inventory_parts ip ON i.id = ip.inventory_id
        WHERE s.num_parts > 0
        GROUP BY s.set_num, s.name, s.year, s.theme_id, s.num_parts, s.img_url, t.name, t.parent_id
        ORDER BY s.set_num;
        """


# ========================================================================================
class ContentBasedRecommender:
    """recommendation_system.py:78-276"""

    def __init__(self, dbcon, engine: Optional[Engine] = None):
        from sklearn.preprocessing import StandardScaler
        self.dbcon = dbcon
        self.engine = engine if engine is not None else Engine(dbcon)
        self.set_feat: Optional[pd.DataFrame] = None
        self.scaler = StandardScaler()
        self.feat_matrix: Optional[np.ndarray] = None
        self.set_lookup: Dict[int, str] = {}
        self._row_of_set: Dict[str, int] = {}
        self._content_row: Optional[np.ndarray] = None   # catalogue row -> set_feat row (-1)

    # ---------------------------------------------------------------- features (:91-192)
    def prepare_features(self):
        logger.info("Preparing content-based features")
        self.set_feat = _read_sql(_FEATURE_SQL, self.dbcon)
        for c in ("num_parts", "unique_parts", "unique_colors", "avg_part_quantity"):
            self.set_feat[c] = self.set_feat[c].fillna(0)
        self.set_feat["complexity_score"] = self._calculate_complexity_score()
        self.set_feat["age_score"] = self._calculate_age_score()
        self.set_feat["size_category"] = self._categorize_by_size()
        self._create_feature_matrix()
        self.set_lookup = dict(zip(range(len(self.set_feat)), self.set_feat["set_num"]))
        self._row_of_set = {s: i for i, s in enumerate(self.set_feat["set_num"])}
        self.engine.set_content(list(self.set_feat["set_num"]), self.feat_matrix)
        cat = self.engine.catalog
        self._content_row = np.full(cat.n, -1, np.int64)
        self._content_row[cat.rows_of(self.set_feat["set_num"])] = np.arange(len(self.set_feat))
        # reason columns, positional
        sf = self.set_feat
        self._r_theme = sf["theme_id"].to_numpy()
        self._r_theme_name = sf["theme_name"].tolist()
        self._r_size = sf["size_category"].tolist()
        self._r_cx = sf["complexity_score"].to_numpy(np.float64)
        self._r_year = sf["year"].to_numpy()
        logger.info(f"Prepared features for {len(self.set_feat)} sets")

    def _calculate_complexity_score(self) -> pd.Series:
        """:144-151"""
        f = self.set_feat
        c = (0.4 * f["num_parts"] / f["num_parts"].max() +
             0.3 * f["unique_parts"] / f["unique_parts"].max() +
             0.2 * f["unique_colors"] / f["unique_colors"].max() +
             0.1 * f["avg_part_quantity"] / f["avg_part_quantity"].max())
        return c.fillna(0)

    def _calculate_age_score(self) -> pd.Series:
        """:153-159 — newer sets score higher; uses the current year."""
        age = _current_year() - self.set_feat["year"]
        return 1 - (age / age.max())

    def _categorize_by_size(self) -> pd.Series:
        """:161-173"""
        def size_category(p):
            if p < 100:
                return "small"
            if p < 500:
                return "medium"
            if p < 1000:
                return "large"
            return "xl"
        return self.set_feat["num_parts"].apply(size_category)

    def _create_feature_matrix(self):
        """:175-192 — StandardScaler over six numeric columns + size one-hot."""
        cols = ["num_parts", "unique_parts", "unique_colors", "complexity_score", "age_score", "theme_id"]
        scaled = self.scaler.fit_transform(self.set_feat[cols].copy())
        dummies = pd.get_dummies(self.set_feat["size_category"], prefix="size")
        self.feat_matrix = np.hstack([scaled, dummies.values])

    # ---------------------------------------------------------------- search (:194-249)
    def _search_rows(self, row: int, k: int, mask: Optional[np.ndarray]):
        idx = self.engine.ensure_index()
        sc, ids, cnt = idx.search("similar", k, q_items=np.array([row], np.int64), mask=mask)
        c = int(cnt[0])
        return ids[0][:c], sc[0][:c]

    def get_similar_sets(self, set_num: str, top_k: int = 10,
                         valid_set_filter: Optional[List[str]] = None) -> List[RecommendationResult]:
        if self.feat_matrix is None:
            self.prepare_features()
        if set_num not in self._row_of_set:
            logger.error(f"Set {set_num} not found")
            return []
        cat = self.engine.catalog
        return self.similar_by_mask(set_num, top_k, cat.mask_of(valid_set_filter))

    def similar_by_mask(self, set_num: str, top_k: int, mask: Optional[np.ndarray]) -> List[RecommendationResult]:
        """get_similar_sets with the valid filter already a catalogue mask (None = all)."""
        if self.feat_matrix is None:
            self.prepare_features()
        if set_num not in self._row_of_set or top_k <= 0:
            return []
        cat = self.engine.catalog
        t = self._row_of_set[set_num]
        ids, sc = self._search_rows(cat.pos[set_num], top_k, mask)
        out = []
        for gid, s in zip(ids, sc):
            i = int(self._content_row[int(gid)])
            out.append(RecommendationResult(
                set_num=self.set_lookup[i], name=self.set_feat["name"].iat[i], score=float(s),
                reasons=self._generate_content_reasons_rows(i, t),
                theme_name=self._r_theme_name[i], year=int(self._r_year[i]),
                num_parts=int(self.set_feat["num_parts"].iat[i]), img_url=self.set_feat["img_url"].iat[i]))
        return out

    def _generate_content_reasons_rows(self, i: int, t: int) -> List[str]:
        """:251-276 on set_feat rows (i = recommended, t = target)."""
        reasons = []
        if self._r_theme[i] == self._r_theme[t]:
            reasons.append(f"Same theme: {self._r_theme_name[i]}")
        if self._r_size[i] == self._r_size[t]:
            reasons.append(f"Same size category: {self._r_size[i]}")
        if abs(self._r_cx[i] - self._r_cx[t]) < 0.2:
            reasons.append("Similar complexity level")
        if abs(self._r_year[i] - self._r_year[t]) <= 3:
            reasons.append("From similar era")
        return reasons

    def _generate_content_reasons(self, similar_set, target_set_num) -> List[str]:
        """Reference signature (a set_feat row + target set_num)."""
        return self._generate_content_reasons_rows(self._row_of_set[similar_set["set_num"]],
                                                   self._row_of_set[target_set_num])


# ========================================================================================
class CollaborativeFilteringRecommender:
    """recommendation_system.py:278-598"""

    def __init__(self, dbcon, engine: Optional[Engine] = None):
        self.dbcon = dbcon
        self.engine = engine if engine is not None else Engine(dbcon)
        self.user_item_matrix: Optional[pd.DataFrame] = None
        self.svd_model = None
        self.user_profiles = {}
        self.item_lookup = {}
        self.reverse_user_profiles = {}
        self.reverse_item_lookup = {}
        self.user_lookup = {}
        self._rated_rows: Dict[int, np.ndarray] = {}   # user idx -> catalogue rows rated > 0

    def prepare_user_item_matrix(self):
        """:292-338"""
        self._create_synthetic_user_data()
        query = """
        SELECT user_id, set_num, rating, interaction_type, created_at
        FROM user_interactions
        WHERE rating IS NOT NULL
        ORDER BY user_id, set_num;
        """
        try:
            ratings_df = _read_sql(query, self.dbcon)
            if ratings_df.empty:
                logger.info("No user rating data found, creating synthetic data for testing")
                ratings_df = self.synthetic_ratings
        except Exception as e:  # same fallback as the reference
            logger.warning(f"Error loading user ratings: {e}, using synthetic data")
            ratings_df = self.synthetic_ratings
        self.user_item_matrix = ratings_df.pivot_table(index="user_id", columns="set_num", values="rating",
                                                       fill_value=0)
        self.user_lookup = {u: i for i, u in enumerate(self.user_item_matrix.index)}
        self.item_lookup = {s: i for i, s in enumerate(self.user_item_matrix.columns)}
        self.reverse_user_lookup = {i: u for u, i in self.user_lookup.items()}
        self.reverse_item_lookup = {i: s for s, i in self.item_lookup.items()}

    def _create_synthetic_user_data(self):
        """:340-366 — same global-RNG draws (seed 42) as the reference."""
        np.random.seed(42)
        set_nums = _read_sql("SELECT set_num FROM sets LIMIT 100", self.dbcon)["set_num"].tolist()
        data = []
        for user_id in range(1, 51):
            num_ratings = np.random.randint(10, 31)
            rated_sets = np.random.choice(set_nums, num_ratings, replace=False)
            for set_num in rated_sets:
                rating = np.random.choice([3, 4, 5], p=[0.2, 0.3, 0.5])
                data.append({"user_id": user_id, "set_num": set_num, "rating": rating,
                             "interaction_type": "rating", "created_at": datetime.now()})
        self.synthetic_ratings = pd.DataFrame(data)

    def train_svd_model(self, n_components: int = 50):
        """:368-409, then the factors go to the device in catalogue rows."""
        from sklearn.decomposition import TruncatedSVD
        if self.user_item_matrix is None:
            self.prepare_user_item_matrix()
        m = self.user_item_matrix
        if m.shape[0] < 3 or m.shape[1] < 3:
            logger.warning(f"Insufficient data for SVD: {m.shape}")
            self.svd_model = None
            return
        n_components = min(n_components, min(m.shape) - 1)
        if n_components < 2:
            self.svd_model = None
            return
        self.svd_model = TruncatedSVD(n_components=n_components, random_state=42)
        self.user_factors = self.svd_model.fit_transform(m)
        self.item_factors = self.svd_model.components_.T
        cat = self.engine.ensure_catalog()
        cols = list(m.columns)
        self.engine.set_cf(cols, self.item_factors)
        col_rows = cat.rows_of(cols)
        vals = m.to_numpy()
        self._rated_rows = {u: col_rows[vals[u] > 0] for u in range(vals.shape[0])}

    def rated_mask(self, user_idx: int) -> np.ndarray:
        m = np.zeros(self.engine.catalog.n, bool)
        m[self._rated_rows[user_idx]] = True
        return m

    def _lookup(self, user_id):
        """user_lookup holds the pivot's int ids; the API passes str(user_id) (a reference
        bug that always fell to cold start): both spellings resolve here."""
        if user_id in self.user_lookup:
            return self.user_lookup[user_id]
        try:
            return self.user_lookup.get(int(user_id))
        except (TypeError, ValueError):
            return None

    def get_recommendations(self, user_id, top_k: int = 10,
                            valid_set_filter: Optional[List[str]] = None) -> List[RecommendationResult]:
        """:411-483"""
        if self.svd_model is None:
            self.train_svd_model()
        if self.svd_model is None:
            return self._cold_start_recommendations(top_k, valid_set_filter)
        u = self._lookup(user_id)
        if u is None:
            logger.warning(f"User {user_id} not found in user lookup")
            return self._cold_start_recommendations(top_k, valid_set_filter)
        return self.recommend_by_mask(u, top_k, self.engine.catalog.mask_of(valid_set_filter))

    def recommend_by_mask(self, u: int, top_k: int, mask: Optional[np.ndarray]) -> List[RecommendationResult]:
        if top_k <= 0:
            return []
        cat = self.engine.catalog
        idx = self.engine.ensure_index()
        sc, ids, cnt = idx.search("cf", top_k, q_cf=self.user_factors[[u]], excl=self.rated_mask(u)[None, :],
                                  mask=mask)
        out = []
        for gid, s in zip(ids[0][: int(cnt[0])], sc[0][: int(cnt[0])]):
            g = int(gid)
            if g >= cat.n_db:   # _get_set_details finds no row (:470-471): skipped
                continue
            d = cat.details(g)
            out.append(RecommendationResult(
                set_num=d["set_num"], name=d["name"], score=float(s),
                reasons=["Users with similar preferences also liked this set"],
                theme_name=d["theme_name"], year=d["year"], num_parts=d["num_parts"], img_url=d["img_url"]))
        return out

    def _cold_start_recommendations(self, top_k: int, valid_set_filter: Optional[List[str]] = None):
        """:485-533 — popular sets by average rating (SQL, off the device path)."""
        q = """
        SELECT s.set_num, s.name, s.year, s.num_parts, s.img_url, t.name as theme_name,
               AVG(ui.rating) as avg_rating, COUNT(ui.rating) as rating_count
        FROM sets s
        LEFT JOIN themes t ON s.theme_id = t.id
        LEFT JOIN user_interactions ui ON s.set_num = ui.set_num
        WHERE ui.rating IS NOT NULL
        """
        params: list = []
        if valid_set_filter:
            q += " AND s.set_num = ANY(%s)"
            params.append(valid_set_filter)
        q += """
        GROUP BY s.set_num, s.name, s.year, s.num_parts, s.img_url, t.name
        HAVING COUNT(ui.rating) >= 3
        ORDER BY avg_rating DESC, rating_count DESC
        LIMIT %s
        """
        params.append(top_k)
        try:
            df = _read_sql(q, self.dbcon, params)
            return [RecommendationResult(
                set_num=r["set_num"], name=r["name"], score=float(r["avg_rating"]),
                reasons=[f"Popular set with {r['rating_count']} ratings"], theme_name=r["theme_name"],
                year=int(r["year"]), num_parts=int(r["num_parts"]), img_url=r["img_url"])
                for _, r in df.iterrows()]
        except Exception as e:
            logger.error(f"Error getting popular recommendations: {e}")
            return self._get_recent_popular_sets(top_k, valid_set_filter)

    def _get_set_details(self, set_num: str) -> Optional[Dict]:
        cat = self.engine.ensure_catalog()
        i = cat.pos.get(set_num)
        return None if i is None or i >= cat.n_db else cat.details(i)

    def _get_recent_popular_sets(self, top_k: int, valid_set_filter: Optional[List[str]] = None):
        """:552-598"""
        q = """
        SELECT s.set_num, s.name, s.year, s.num_parts, s.img_url, t.name as theme_name
        FROM sets s
        LEFT JOIN themes t ON s.theme_id = t.id
        WHERE s.year >= 2020 AND s.num_parts BETWEEN 100 AND 1000
        """
        params: list = []
        if valid_set_filter:
            q += " AND s.set_num = ANY(%s)"
            params.append(valid_set_filter)
        q += " ORDER BY s.year DESC, s.num_parts DESC LIMIT %s"
        params.append(top_k)
        try:
            df = _read_sql(q, self.dbcon, params)
            return [RecommendationResult(
                set_num=r["set_num"], name=r["name"], score=0.8, reasons=["Popular recent set"],
                theme_name=r["theme_name"] or "Unknown", year=int(r["year"]), num_parts=int(r["num_parts"]),
                img_url=r["img_url"]) for _, r in df.iterrows()]
        except Exception as e:
            logger.error(f"Error getting recent popular sets: {e}")
            return []


# ========================================================================================
class HybridRecommender:
    """recommendation_system.py:600-851"""

    def __init__(self, dbcon, engine: Optional[Engine] = None):
        self.dbcon = dbcon
        self.engine = engine if engine is not None else Engine(dbcon)
        self.content_recommender = ContentBasedRecommender(dbcon, self.engine)
        self.collaborative_recommender = CollaborativeFilteringRecommender(dbcon, self.engine)
        self.constraint_filter = HardConstraintFilter(dbcon, self.engine)
        self.content_weight = 0.4
        self.collaborative_weight = 0.6

    def get_recommendations(self, user_id: Optional[int] = None, liked_set: Optional[str] = None,
                            top_k: int = 10, constraints: Optional[List[HardConstraint]] = None
                            ) -> Tuple[List[RecommendationResult], Optional[ConstraintResult]]:
        """:612-677"""
        constraint_result = None
        valid = None
        mask = None
        if constraints:
            constraint_result = self.constraint_filter.apply_constraints(constraints)
            valid = constraint_result.valid_set_nums
            if not valid:
                logger.warning("No sets meet the specified hard constraints")
                return [], constraint_result
            mask = constraint_result.valid_mask
        content_recs: List[RecommendationResult] = []
        collaborative_recs: List[RecommendationResult] = []
        fused = self._device_hybrid(user_id, liked_set, top_k, self._mask_for(mask))
        if fused is not None:
            if constraint_result and constraint_result.violations:
                for rec in fused:
                    rec.constraint_violations = [v.message for v in constraint_result.violations]
            return fused, constraint_result
        if liked_set:
            cr = self.content_recommender
            if cr.feat_matrix is None:
                cr.prepare_features()
            if liked_set in cr._row_of_set:
                content_recs = cr.similar_by_mask(liked_set, top_k * 2, self._mask_for(mask))
            else:
                logger.error(f"Set {liked_set} not found")
        if user_id:
            cf = self.collaborative_recommender
            if cf.svd_model is None:
                cf.train_svd_model()
            u = cf._lookup(user_id) if cf.svd_model is not None else None
            if u is not None:
                collaborative_recs = cf.recommend_by_mask(u, top_k * 2, self._mask_for(mask))
            else:
                collaborative_recs = cf._cold_start_recommendations(top_k * 2, valid)
        if not content_recs and collaborative_recs:
            final = collaborative_recs[:top_k]
        elif content_recs and not collaborative_recs:
            final = content_recs[:top_k]
        elif not content_recs and not collaborative_recs:
            final = self._get_constrained_popular_sets(top_k, valid)
        else:
            final = self._combine_recommendations(content_recs, collaborative_recs, top_k)
        if constraint_result and constraint_result.violations:
            for rec in final:
                rec.constraint_violations = [v.message for v in constraint_result.violations]
        return final, constraint_result

    def _device_hybrid(self, user_id, liked_set, top_k: int, mask: Optional[np.ndarray]
                       ) -> Optional[List[RecommendationResult]]:
        """Both sides available (a known liked set and a user the CF model knows): the whole
        hybrid — content top-2k, CF top-2k, union blend (:646-668, :789-843) — in ONE device
        HYBRID search (bb_search + bb_finalize); reasons follow each item's side membership
        as in _combine_recommendations.  None = take the per-side path (a side is missing,
        a cold-start user, or a CF-side set without a catalogue row, which the reference's
        _get_set_details would drop, :470-471)."""
        if not liked_set or not user_id or top_k <= 0:
            return None
        cr, cf = self.content_recommender, self.collaborative_recommender
        if cr.feat_matrix is None:
            cr.prepare_features()
        if liked_set not in cr._row_of_set:
            return None
        if cf.svd_model is None:
            cf.train_svd_model()
        u = cf._lookup(user_id) if cf.svd_model is not None else None
        if u is None:
            return None
        cat = self.engine.catalog
        idx = self.engine.ensure_index()
        sc, ids, cnt, in_c, in_f, sides = idx.search_hybrid_sides(
            top_k, q_items=[cat.pos[liked_set]], q_cf=cf.user_factors[[u]], excl=cf.rated_mask(u)[None, :],
            mask=mask, w_content=self.content_weight, w_cf=self.collaborative_weight)
        c_ids, f_ids = sides[0]
        if len(f_ids) and int(np.max(f_ids)) >= cat.n_db:
            return None
        if len(c_ids) == 0 or len(f_ids) == 0:
            # one side produced nothing: the reference then takes the other side's top k with
            # its own scores (:659-662), which the per-side path reproduces
            return None
        t = cr._row_of_set[liked_set]
        out = []
        for j in range(int(cnt[0])):
            g = int(ids[0][j])
            reasons = []
            if in_c[0][j]:
                i = int(cr._content_row[g])
                reasons += [f"Content: {x}" for x in cr._generate_content_reasons_rows(i, t)]
                base = dict(set_num=cr.set_lookup[i], name=cr.set_feat["name"].iat[i],
                            theme_name=cr._r_theme_name[i], year=int(cr._r_year[i]),
                            num_parts=int(cr.set_feat["num_parts"].iat[i]), img_url=cr.set_feat["img_url"].iat[i])
            else:
                d = cat.details(g)
                base = dict(set_num=d["set_num"], name=d["name"], theme_name=d["theme_name"], year=d["year"],
                            num_parts=d["num_parts"], img_url=d["img_url"])
            if in_f[0][j]:
                reasons.append("Community: Users with similar preferences also liked this set")
            out.append(RecommendationResult(score=float(sc[0][j]), reasons=reasons, **base))
        return out

    def _mask_for(self, mask: Optional[np.ndarray]) -> Optional[np.ndarray]:
        """Pad a constraint mask to the current catalogue size (rows appended since)."""
        if mask is None:
            return None
        n = self.engine.catalog.n
        if len(mask) == n:
            return mask
        out = np.zeros(n, bool)
        out[: len(mask)] = mask
        return out

    def get_recommendations_from_request(self, request: RecommendationRequest
                                         ) -> Tuple[List[RecommendationResult], ConstraintResult]:
        """:679-719"""
        try:
            constraints = self.constraint_filter.create_constraint_set(
                price_max=request.price_max, price_min=request.price_min, pieces_max=request.pieces_max,
                pieces_min=request.pieces_min, age_min=request.age_min, age_max=request.age_max,
                year_min=request.year_min, year_max=request.year_max, required_themes=request.required_themes,
                excluded_themes=request.excluded_themes, max_complexity=request.max_complexity,
                min_complexity=request.min_complexity, must_be_available=request.must_be_available,
                exclude_owned=request.exclude_owned, exclude_wishlisted=request.exclude_wishlisted,
                user_id=request.user_id)
        except Exception as e:
            logger.error(f"Failed to create constraints: {e}")
            return [], ConstraintResult(valid_set_nums=[], violations=[], applied_constraints=[],
                                        performance_stats={})
        return self.get_recommendations(user_id=request.user_id, liked_set=request.liked_set,
                                        top_k=request.top_k, constraints=constraints)

    def _get_constrained_popular_sets(self, top_k: int, valid_set_nums: Optional[List[str]] = None):
        """:721-787 (SQL, off the device path)."""
        q = """
        SELECT s.set_num, s.name, s.year, s.num_parts, s.img_url, t.name as theme_name,
               COALESCE(AVG(ui.rating), 0) as avg_rating,
               COUNT(ui.rating) as rating_count,
               s.year as popularity_boost
        FROM sets s
        LEFT JOIN themes t ON s.theme_id = t.id
        LEFT JOIN user_interactions ui ON s.set_num = ui.set_num AND ui.rating IS NOT NULL
        WHERE s.num_parts > 0
        """
        params: list = []
        if valid_set_nums:
            q += f" AND s.set_num IN ({','.join(['%s'] * len(valid_set_nums))})"
            params.extend(valid_set_nums)
        q += """
        GROUP BY s.set_num, s.name, s.year, s.num_parts, s.img_url, t.name
        ORDER BY
            CASE WHEN COUNT(ui.rating) >= 3 THEN AVG(ui.rating) ELSE 0 END DESC,
            COUNT(ui.rating) DESC,
            s.year DESC
        LIMIT %s
        """
        params.append(top_k)
        try:
            df = _read_sql(q, self.dbcon, params)
            out = []
            for _, r in df.iterrows():
                reasons = ["Popular choice"]
                if r["rating_count"] > 0:
                    reasons.append(f"Avg rating: {r['avg_rating']:.1f} ({r['rating_count']} reviews)")
                else:
                    reasons.append("Recent release")
                out.append(RecommendationResult(
                    set_num=r["set_num"], name=r["name"],
                    score=float(r["avg_rating"]) if r["rating_count"] > 0 else 0.5, reasons=reasons,
                    theme_name=r["theme_name"], year=int(r["year"]), num_parts=int(r["num_parts"]),
                    img_url=r["img_url"]))
            return out
        except Exception as e:
            logger.error(f"Error getting constrained popular sets: {e}")
            return []

    def _combine_recommendations(self, content_recs: List[RecommendationResult],
                                 collaborative_recs: List[RecommendationResult], top_k: int
                                 ) -> List[RecommendationResult]:
        """:789-843 — union blend, missing side = 0, f64; ties by catalogue row."""
        cd = {r.set_num: r for r in content_recs}
        fd = {r.set_num: r for r in collaborative_recs}
        pos = self.engine.ensure_catalog().pos
        combined = []
        for s in set(cd) | set(fd):
            c, f = cd.get(s), fd.get(s)
            h = self.content_weight * (c.score if c else 0) + self.collaborative_weight * (f.score if f else 0)
            base = c if c else f
            reasons = [f"Content: {x}" for x in (c.reasons if c else [])]
            reasons += [f"Community: {x}" for x in (f.reasons if f else [])]
            combined.append(RecommendationResult(set_num=s, name=base.name, score=h, reasons=reasons,
                                                 theme_name=base.theme_name, year=base.year,
                                                 num_parts=base.num_parts, img_url=base.img_url))
        combined.sort(key=lambda r: (-r.score, pos.get(r.set_num, 1 << 62)))
        return combined[:top_k]

    def set_weights(self, content_weight: float, collaborative_weight: float):
        """:845-851"""
        total = content_weight + collaborative_weight
        self.content_weight = content_weight / total
        self.collaborative_weight = collaborative_weight / total

    # ---------------------------------------------------------------- batched device path
    def recommend_batch(self, liked_sets: Sequence[Optional[str]], user_ids: Sequence[Optional[int]],
                        top_k: int = 10, mask: Optional[np.ndarray] = None):
        """Many hybrid queries in ONE device call: content top-2k ∪ CF top-2k, blended on the
        device (bb_search HYBRID).  Every query needs a known liked set and a known user
        (the single-sided and cold-start cases are per-request in get_recommendations).
        Returns (set_nums [B][<=k], scores [B][<=k])."""
        cr, cf = self.content_recommender, self.collaborative_recommender
        if cr.feat_matrix is None:
            cr.prepare_features()
        if cf.svd_model is None:
            cf.train_svd_model()
        cat = self.engine.catalog
        rows = np.array([cat.pos[s] for s in liked_sets], np.int64)
        us = [cf._lookup(u) for u in user_ids]
        if any(u is None for u in us):
            raise KeyError("recommend_batch: every user must be known to the CF model")
        excl = np.stack([cf.rated_mask(u) for u in us])
        sc, ids, cnt = self.engine.ensure_index().search(
            "hybrid", top_k, q_items=rows, q_cf=cf.user_factors[us], excl=excl, mask=self._mask_for(mask),
            w_content=self.content_weight, w_cf=self.collaborative_weight)
        names = [[cat.set_nums[int(g)] for g in ids[b][: int(cnt[b])]] for b in range(len(rows))]
        return names, [sc[b][: int(cnt[b])] for b in range(len(rows))]
