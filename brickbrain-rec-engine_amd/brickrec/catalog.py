"""The catalogue: one item space shared by the content, CF and constraint drop-ins.

Rows are every set of the ``sets`` table ordered by ``set_num``.  That order is the order the
content features use (recommendation_system.py:117, ``ORDER BY s.set_num``), so the content
rows are a subsequence of it (``WHERE s.num_parts > 0``).  The CF pivot columns
(``:325-336``) map into it by set_num too.  Sets that only the ratings know are appended.
The device index (``Engine.index``) is laid out in this order:

* content feature rows (present bits = the content item space);
* CF item factors (present bits = the pivot columns);
* the attribute columns that the hard-constraint predicates read
  (hard_constraint_filter.py:366-480).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, List, Optional, Sequence, Set

import numpy as np


def query_rows(dbcon, sql: str, params: Sequence[Any] = ()) -> List[Dict[str, Any]]:
    """Run one query on a DB-API connection (psycopg2 or a compatible wrapper); dict rows."""
    cur = dbcon.cursor()
    try:
        cur.execute(sql, list(params))
        cols = [d[0] for d in cur.description]
        out = []
        for r in cur.fetchall():
            out.append(dict(r) if isinstance(r, dict) else dict(zip(cols, r)))
        return out
    finally:
        try:
            cur.close()
        except Exception:
            pass


@dataclass
class Catalog:
    set_nums: List[str]
    name: List[str]
    year: np.ndarray          # int64
    theme_id: np.ndarray      # int64, -1 = NULL
    num_parts: np.ndarray     # int64
    img_url: List[Optional[str]]
    theme_name: List[Optional[str]]
    theme_names: Dict[int, str] = field(default_factory=dict)
    pos: Dict[str, int] = field(default_factory=dict)
    n_db: int = -1            # rows that come from the sets table (the rest were appended)

    def __post_init__(self):
        if not self.pos:
            self.pos = {s: i for i, s in enumerate(self.set_nums)}
        if self.n_db < 0:
            self.n_db = len(self.set_nums)

    @property
    def n(self) -> int:
        return len(self.set_nums)

    @classmethod
    def from_db(cls, dbcon) -> "Catalog":
        rows = query_rows(dbcon, """
            SELECT s.set_num, s.name, s.year, s.theme_id, s.num_parts, s.img_url, t.name AS theme_name
            FROM sets s LEFT JOIN themes t ON s.theme_id = t.id
            ORDER BY s.set_num""")
        themes = query_rows(dbcon, "SELECT id, name FROM themes")
        return cls(
            set_nums=[r["set_num"] for r in rows],
            name=[r["name"] for r in rows],
            year=np.array([int(r["year"]) if r["year"] is not None else 0 for r in rows], np.int64),
            theme_id=np.array([int(r["theme_id"]) if r["theme_id"] is not None else -1 for r in rows], np.int64),
            num_parts=np.array([int(r["num_parts"]) if r["num_parts"] is not None else 0 for r in rows], np.int64),
            img_url=[r["img_url"] for r in rows],
            theme_name=[r["theme_name"] for r in rows],
            theme_names={int(t["id"]): t["name"] for t in themes},
        )

    def extend(self, set_nums: Iterable[str]) -> List[int]:
        """Append sets the catalogue does not hold (e.g. rated sets missing from ``sets``)."""
        added = []
        for s in set_nums:
            if s not in self.pos:
                self.pos[s] = len(self.set_nums)
                self.set_nums.append(s)
                self.name.append(s)
                self.img_url.append(None)
                self.theme_name.append(None)
                added.append(self.pos[s])
        if added:
            k = len(added)
            self.year = np.concatenate([self.year, np.zeros(k, np.int64)])
            self.theme_id = np.concatenate([self.theme_id, np.full(k, -1, np.int64)])
            self.num_parts = np.concatenate([self.num_parts, np.zeros(k, np.int64)])
        return added

    def rows_of(self, set_nums: Iterable[str]) -> np.ndarray:
        return np.array([self.pos[s] for s in set_nums if s in self.pos], np.int64)

    def mask_of(self, set_nums: Optional[Iterable[str]]) -> Optional[np.ndarray]:
        """valid_set_filter -> bool mask; None or an empty list means "no filter", as the
        reference's ``if valid_set_filter and ...`` tests (recommendation_system.py:229, 454)."""
        if not set_nums:
            return None
        m = np.zeros(self.n, bool)
        m[self.rows_of(set_nums)] = True
        return m

    def user_sets(self, dbcon, table: str, user_id) -> Set[int]:
        """Rows of a user's collection / wishlist (the NOT EXISTS subqueries of
        hard_constraint_filter.py:441-451)."""
        if table not in ("user_collections", "user_wishlists"):
            raise ValueError(table)
        rows = query_rows(dbcon, f"SELECT set_num FROM {table} WHERE user_id = %s", [user_id])
        return {self.pos[r["set_num"]] for r in rows if r["set_num"] in self.pos}

    def details(self, i: int) -> Dict[str, Any]:
        """``_get_set_details`` (recommendation_system.py:535-550) without a query per row."""
        return {"set_num": self.set_nums[i], "name": self.name[i], "year": int(self.year[i]),
                "num_parts": int(self.num_parts[i]), "img_url": self.img_url[i],
                "theme_name": self.theme_name[i]}


class Engine:
    """Catalogue + one device index shared by the recommenders of one process.

    ``index_factory(n)`` builds the device index.  It defaults to
    :class:`brickrec.engine.ItemIndex`, and tests may inject another one.  The drop-ins
    call ``ensure_*`` lazily, so a recommender works on its own as in the reference, and
    the three drop-ins of a ``HybridRecommender`` share one catalogue and one index.
    """

    def __init__(self, dbcon, device: int = 0, dtype: str = "f32", index_factory=None):
        self.dbcon = dbcon
        self.device = device
        self.dtype = dtype
        self._factory = index_factory
        self._mu = threading.RLock()
        self.catalog: Optional[Catalog] = None
        self.index = None
        self.content_present: Optional[np.ndarray] = None
        self.cf_present: Optional[np.ndarray] = None
        self._features: Optional[np.ndarray] = None      # [n, F] f64 in catalogue rows
        self._factors: Optional[np.ndarray] = None       # [n, r] in catalogue rows
        self.version = 0                                 # bumps on every device upload

    def ensure_catalog(self) -> Catalog:
        with self._mu:
            if self.catalog is None:
                self.catalog = Catalog.from_db(self.dbcon)
            return self.catalog

    def _new_index(self):
        if self._factory is not None:
            return self._factory()
        from .engine import ItemIndex
        return ItemIndex(device=self.device, dtype=self.dtype)

    def _upload(self):
        """(Re)build the device copy: items (features or a zero column), attrs, CF factors."""
        cat = self.catalog
        n = cat.n
        if self.index is None:
            self.index = self._new_index()
        if self._features is not None:
            feats = np.zeros((n, self._features.shape[1]))
            feats[: self._features.shape[0]] = self._features
            self.index.upload_items(feats, present=self._pad(self.content_present, n))
        else:
            self.index.upload_items(np.zeros((n, 4)), present=np.zeros(n, bool))
        self.index.upload_attrs(cat.num_parts.astype(np.int32),
                                np.clip(cat.year, -32768, 32767).astype(np.int16),
                                cat.theme_id.astype(np.int32))
        if self._factors is not None:
            f = np.zeros((n, self._factors.shape[1]))
            f[: self._factors.shape[0]] = self._factors
            self.index.upload_cf(f, present=self._pad(self.cf_present, n))
        self.version += 1

    @staticmethod
    def _pad(m, n):
        out = np.zeros(n, bool)
        if m is not None:
            out[: len(m)] = m
        return out

    def ensure_index(self):
        with self._mu:
            self.ensure_catalog()
            if self.index is None:
                self._upload()
            return self.index

    def set_content(self, set_nums: Sequence[str], feat_matrix: np.ndarray):
        """Content rows (set_feat order) -> catalogue rows; upload."""
        with self._mu:
            cat = self.ensure_catalog()
            cat.extend(set_nums)
            rows = cat.rows_of(set_nums)
            F = np.zeros((cat.n, feat_matrix.shape[1]))
            F[rows] = feat_matrix
            present = np.zeros(cat.n, bool)
            present[rows] = True
            self._features, self.content_present = F, present
            self._upload()

    def set_cf(self, columns: Sequence[str], item_factors: np.ndarray):
        """CF pivot columns -> catalogue rows; upload."""
        with self._mu:
            cat = self.ensure_catalog()
            cat.extend(columns)
            rows = cat.rows_of(columns)
            F = np.zeros((cat.n, item_factors.shape[1]))
            F[rows] = item_factors
            present = np.zeros(cat.n, bool)
            present[rows] = True
            self._factors, self.cf_present = F, present
            self._upload()
