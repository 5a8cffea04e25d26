"""Hard-constraint filtering — drop-in for ``src/scripts/hard_constraint_filter.py``.

Same public names and behaviour (``ConstraintType``, ``HardConstraint``,
``ConstraintResult``, ``HardConstraintFilter.create_constraint_set`` /
``apply_constraints`` ...), but the WHERE clause of ``_build_constraint_sql``
(hard_constraint_filter.py:318-480) is compiled into a :class:`~brickrec.engine.Predicate`
and evaluated on the GPU over the catalogue's attribute columns (``bb_eval_mask``),
instead of one SQL query plus one more per constraint for the diagnostics (:281-288,
:564-568).  Only the owned/wishlisted sets of the requesting user are still read from
the database (one small query each, the NOT EXISTS of :441-451).
"""
from __future__ import annotations

import logging
import re
import time
from dataclasses import dataclass, field
from datetime import datetime
from enum import Enum
from typing import Any, Dict, Iterable, List, Optional, Sequence, Set, Tuple

import numpy as np

from .engine import INT32_MAX, INT32_MIN, Predicate

logger = logging.getLogger(__name__)


class ConstraintType(Enum):
    """hard_constraint_filter.py:14-30"""
    PRICE_MAX = "price_max"
    PRICE_MIN = "price_min"
    PIECES_MAX = "pieces_max"
    PIECES_MIN = "pieces_min"
    AGE_MIN = "age_min"
    AGE_MAX = "age_max"
    YEAR_MIN = "year_min"
    YEAR_MAX = "year_max"
    THEMES_REQUIRED = "themes_required"
    THEMES_EXCLUDED = "themes_excluded"
    COMPLEXITY_MAX = "complexity_max"
    COMPLEXITY_MIN = "complexity_min"
    AVAILABILITY = "availability"
    EXCLUDE_OWNED = "exclude_owned"
    EXCLUDE_WISHLISTED = "exclude_wishlisted"


class ConstraintSeverity(Enum):
    """:32-36"""
    BLOCKING = "blocking"
    WARNING = "warning"
    INFO = "info"


@dataclass
class HardConstraint:
    """:38-48"""
    constraint_type: ConstraintType
    value: Any
    severity: ConstraintSeverity = ConstraintSeverity.BLOCKING
    description: str = ""

    def __post_init__(self):
        if not self.description:
            self.description = f"{self.constraint_type.value}: {self.value}"


@dataclass
class ConstraintViolation:
    """:50-57"""
    constraint: HardConstraint
    violating_count: int
    total_count: int
    message: str
    suggested_alternatives: List[str] = None


@dataclass
class ConstraintResult:
    """:59-66"""
    valid_set_nums: List[str]
    violations: List[ConstraintViolation]
    applied_constraints: List[HardConstraint]
    performance_stats: Dict[str, Any]
    constraint_sql: str = ""
    valid_mask: Optional[np.ndarray] = field(default=None, repr=False)  # bool over the catalogue


def create_constraint_set_values(price_max=None, price_min=None, pieces_max=None, pieces_min=None,
                                 age_min=None, age_max=None, year_min=None, year_max=None,
                                 required_themes=None, excluded_themes=None, max_complexity=None,
                                 min_complexity=None, must_be_available=False, exclude_owned=False,
                                 exclude_wishlisted=False, user_id=None) -> List[HardConstraint]:
    """``create_constraint_set`` (:98-261): same order, same descriptions, same
    user_id-less warnings for the personal constraints."""
    c: List[HardConstraint] = []
    T = ConstraintType
    if price_max is not None:
        c.append(HardConstraint(T.PRICE_MAX, price_max, description=f"Must cost less than ${price_max:.2f}"))
    if price_min is not None:
        c.append(HardConstraint(T.PRICE_MIN, price_min, description=f"Must cost more than ${price_min:.2f}"))
    if pieces_max is not None:
        c.append(HardConstraint(T.PIECES_MAX, pieces_max, description=f"Must have fewer than {pieces_max} pieces"))
    if pieces_min is not None:
        c.append(HardConstraint(T.PIECES_MIN, pieces_min, description=f"Must have more than {pieces_min} pieces"))
    if age_min is not None:
        c.append(HardConstraint(T.AGE_MIN, age_min, description=f"Must be suitable for ages {age_min}+"))
    if age_max is not None:
        c.append(HardConstraint(T.AGE_MAX, age_max, description=f"Must be suitable for ages up to {age_max}"))
    if year_min is not None:
        c.append(HardConstraint(T.YEAR_MIN, year_min, description=f"Must be released after {year_min}"))
    if year_max is not None:
        c.append(HardConstraint(T.YEAR_MAX, year_max, description=f"Must be released before {year_max}"))
    if required_themes:
        c.append(HardConstraint(T.THEMES_REQUIRED, required_themes,
                                description=f"Must be from themes: {', '.join(required_themes)}"))
    if excluded_themes:
        c.append(HardConstraint(T.THEMES_EXCLUDED, excluded_themes,
                                description=f"Must NOT be from themes: {', '.join(excluded_themes)}"))
    if max_complexity:
        c.append(HardConstraint(T.COMPLEXITY_MAX, max_complexity,
                                description=f"Must be {max_complexity} complexity or simpler"))
    if min_complexity:
        c.append(HardConstraint(T.COMPLEXITY_MIN, min_complexity,
                                description=f"Must be {min_complexity} complexity or more complex"))
    if exclude_owned:
        if not user_id:
            logger.warning("exclude_owned requires user_id, constraint will be ignored")
        else:
            c.append(HardConstraint(T.EXCLUDE_OWNED, user_id, description="Must not be in user's collection"))
    if exclude_wishlisted:
        if not user_id:
            logger.warning("exclude_wishlisted requires user_id, constraint will be ignored")
        else:
            c.append(HardConstraint(T.EXCLUDE_WISHLISTED, user_id, description="Must not be in user's wishlist"))
    if must_be_available:
        c.append(HardConstraint(T.AVAILABILITY, True, description="Must be currently available for purchase"))
    return c


def _like_regex(pattern: str) -> "re.Pattern":
    """SQL LIKE -> regex (``%`` any run, ``_`` one char)."""
    return re.compile("".join(".*" if ch == "%" else "." if ch == "_" else re.escape(ch) for ch in pattern),
                      re.DOTALL)


def theme_ids_like(theme_names: Dict[int, str], names: Iterable[str], exact_match: bool = False) -> List[int]:
    """``_get_theme_ids`` (:482-532): ``LOWER(name) LIKE LOWER('%n%')`` OR-ed over names."""
    if exact_match:
        want = {n.lower() for n in names}
        return sorted(t for t, tn in theme_names.items() if tn is not None and tn.lower() in want)
    pats = [_like_regex(f"%{n}%".lower()) for n in names]
    return sorted(t for t, tn in theme_names.items()
                  if tn is not None and any(p.fullmatch(tn.lower()) for p in pats))


def _ctype(c) -> Tuple[str, Any]:
    if isinstance(c, HardConstraint):
        return c.constraint_type.value, c.value
    return c[0], c[1]


def predicate_from_constraints(constraints: Sequence, theme_names: Dict[int, str],
                               owned: Dict[Any, Set[int]], wishlisted: Dict[Any, Set[int]],
                               current_year: Optional[int] = None) -> Optional[Predicate]:
    """Compile ``_constraint_to_sql`` (:366-480) into one conjunctive Predicate.

    Returns None when the conjunction is unsatisfiable by construction (the ``1=0`` of a
    required theme with no match, :409).  owned / wishlisted map user_id -> item ids."""
    if current_year is None:
        current_year = datetime.now().year
    p = Predicate()
    lo_p, hi_p, lo_y, hi_y = INT32_MIN, INT32_MAX, INT32_MIN, INT32_MAX
    required: Optional[Set[int]] = None
    excluded: Set[int] = set()
    ex_items: Set[int] = set()

    def parts_le(v):
        nonlocal hi_p
        hi_p = min(hi_p, int(v))

    def parts_ge(v):
        nonlocal lo_p
        lo_p = max(lo_p, int(v))

    for c in constraints:
        t, v = _ctype(c)
        if t == "pieces_max":
            parts_le(v)
        elif t == "pieces_min":
            parts_ge(v)
        elif t == "year_min":
            lo_y = max(lo_y, int(v))
        elif t == "year_max":
            hi_y = min(hi_y, int(v))
        elif t == "price_max":
            parts_le(int(v / 0.10))
        elif t == "price_min":
            parts_ge(int(v / 0.15))
        elif t == "themes_required":
            ids = set(theme_ids_like(theme_names, v))
            if not ids:
                return None
            required = ids if required is None else required & ids
        elif t == "themes_excluded":
            excluded |= set(theme_ids_like(theme_names, v))
        elif t == "age_min":
            if v <= 4:
                parts_le(50)
            elif v <= 8:
                parts_le(500)
            elif v <= 12:
                parts_le(1500)
            else:
                parts_ge(500)
        elif t == "age_max":
            if v <= 8:
                parts_le(300)
            elif v <= 12:
                parts_le(800)
        elif t == "exclude_owned":
            ex_items |= set(owned.get(v, ()))
        elif t == "exclude_wishlisted":
            ex_items |= set(wishlisted.get(v, ()))
        elif t == "complexity_max":
            parts_le({"simple": 200, "moderate": 800, "complex": 999999}.get(v, 999999))
        elif t == "complexity_min":
            parts_ge({"simple": 0, "moderate": 200, "complex": 800}.get(v, 0))
        elif t == "availability":
            lo_y = max(lo_y, current_year - 5)
    p.parts_min, p.parts_max, p.year_min, p.year_max = lo_p, hi_p, lo_y, hi_y
    if required is not None:
        p.theme_mode, p.theme_ids = 1, sorted(required - excluded)
    elif excluded:
        p.theme_mode, p.theme_ids = 2, sorted(excluded)
    p.excluded_items = sorted(ex_items)
    return p


def _suggestions(constraint: HardConstraint) -> List[str]:
    """``_generate_constraint_alternatives`` (:590-639)."""
    t, v = constraint.constraint_type, constraint.value
    T = ConstraintType
    s: List[str] = []
    if t == T.PIECES_MAX:
        s = [f"Try increasing to {int(v * 1.5)} pieces", f"Consider {int(v * 2)} pieces for more options",
             "Remove piece count limit and use price instead"]
    elif t == T.PIECES_MIN:
        s = [f"Try decreasing to {int(v * 0.7)} pieces", f"Consider {int(v * 0.5)} pieces for more options",
             "Remove minimum piece requirement"]
    elif t == T.PRICE_MAX:
        s = [f"Try increasing budget to ${v * 1.3:.2f}", f"Consider ${v * 1.5:.2f} for more premium options",
             "Look for sales or discounted sets"]
    elif t == T.THEMES_REQUIRED:
        s = ["Try broader theme categories (e.g., 'space' instead of 'Star Wars')", "Consider related themes",
             "Remove theme restriction and browse by interest category"]
    elif t == T.AGE_MIN:
        s = [f"Try age {v - 2}+ for more options", "Consider that age ratings are conservative",
             "Look at similar complexity levels across age ranges"]
    return s[:3]


class HardConstraintFilter:
    """Drop-in for ``HardConstraintFilter`` (hard_constraint_filter.py:68-662).

    ``engine`` is the shared :class:`brickrec.catalog.Engine` (catalogue + device index with
    the attribute columns); one is built from ``dbcon`` when not given."""

    def __init__(self, dbcon, engine=None):
        from .catalog import Engine
        self.dbcon = dbcon
        self.engine = engine if engine is not None else Engine(dbcon)
        self._theme_cache: Dict[tuple, List[int]] = {}
        self.performance_stats = {'total_constraints_applied': 0, 'total_sets_filtered': 0,
                                  'average_filter_time_ms': 0, 'constraint_hit_rates': {}}

    @property
    def catalog(self):
        return self.engine.ensure_catalog()

    def create_constraint_set(self, **kw) -> List[HardConstraint]:
        return create_constraint_set_values(**kw)

    def _get_theme_ids(self, theme_names: List[str], exact_match: bool = False) -> List[int]:
        key = tuple(sorted(theme_names))
        if key not in self._theme_cache:
            self._theme_cache[key] = theme_ids_like(self.catalog.theme_names, theme_names, exact_match)
        return self._theme_cache[key]

    def _mask(self, constraints: Sequence[HardConstraint]) -> np.ndarray:
        cat = self.catalog
        users = {c.value for c in constraints
                 if c.constraint_type in (ConstraintType.EXCLUDE_OWNED, ConstraintType.EXCLUDE_WISHLISTED)}
        owned = {u: cat.user_sets(self.dbcon, "user_collections", u) for u in users}
        wished = {u: cat.user_sets(self.dbcon, "user_wishlists", u) for u in users}
        pred = predicate_from_constraints(constraints, cat.theme_names, owned, wished)
        if pred is None:
            return np.zeros(cat.n, dtype=bool)
        return self.engine.ensure_index().eval_mask(pred)

    def apply_constraints(self, constraints: List[HardConstraint],
                          candidate_set_nums: Optional[List[str]] = None) -> ConstraintResult:
        """:263-316 — valid sets ordered by set_num, plus the >80 %-elimination
        diagnostics of :534-588 computed from one device mask per constraint."""
        t0 = time.perf_counter()
        cat = self.catalog
        cand = None
        if candidate_set_nums:
            cand = np.zeros(cat.n, dtype=bool)
            cand[[cat.pos[s] for s in candidate_set_nums if s in cat.pos]] = True
        m = self._mask(constraints)
        if cand is not None:
            m &= cand
        valid = [cat.set_nums[i] for i in np.flatnonzero(m)]
        violations = []
        base = cat.num_parts > 0
        if cand is not None:
            base &= cand
        total = int(base.sum())
        for c in constraints:
            single = self._mask([c])
            if cand is not None:
                single &= cand
            remaining = int(single.sum())
            rate = (total - remaining) / total if total else 0.0
            if rate > 0.8:
                violations.append(ConstraintViolation(
                    constraint=c, violating_count=total - remaining, total_count=total,
                    message=f"Constraint '{c.description}' eliminated {rate:.1%} of sets",
                    suggested_alternatives=_suggestions(c)))
        ms = (time.perf_counter() - t0) * 1000
        self._update_performance_stats(len(constraints), len(valid), ms)
        return ConstraintResult(
            valid_set_nums=valid, violations=violations, applied_constraints=constraints,
            performance_stats={'filter_time_ms': ms,
                               'input_sets': len(candidate_set_nums) if candidate_set_nums else 'all',
                               'output_sets': len(valid), 'constraint_count': len(constraints)},
            constraint_sql="device predicate: " + repr(predicate_from_constraints(
                constraints, cat.theme_names, {}, {})), valid_mask=m)

    def _update_performance_stats(self, constraint_count: int, result_count: int, filter_time: float):
        st = self.performance_stats
        st['total_constraints_applied'] += constraint_count
        st['total_sets_filtered'] += result_count
        n = st.get('operation_count', 0) + 1
        st['average_filter_time_ms'] = (st['average_filter_time_ms'] * (n - 1) + filter_time) / n
        st['operation_count'] = n

    def get_performance_report(self) -> Dict[str, Any]:
        return self.performance_stats.copy()

    def clear_cache(self):
        self._theme_cache.clear()


def create_budget_constraints(budget_max: float, budget_min: float = None) -> List[HardConstraint]:
    """:663-678"""
    c = []
    if budget_max is not None:
        c.append(HardConstraint(ConstraintType.PRICE_MAX, budget_max, description=f"Budget limit: ${budget_max:.2f}"))
    if budget_min is not None:
        c.append(HardConstraint(ConstraintType.PRICE_MIN, budget_min, description=f"Budget floor: ${budget_min:.2f}"))
    return c


def create_age_appropriate_constraints(age: int, strict: bool = True) -> List[HardConstraint]:
    """:694-713"""
    v = max(4, age - 2) if strict else max(4, age - 4)
    kind = "strict" if strict else "flexible"
    return [HardConstraint(ConstraintType.AGE_MIN, v, description=f"Age appropriate for {age} year old ({kind})")]


def create_size_constraints(size_category: str) -> List[HardConstraint]:
    """:715-740"""
    ranges = {'mini': (1, 50), 'small': (51, 200), 'medium': (201, 800), 'large': (801, 2000), 'xl': (2001, 10000)}
    if size_category.lower() not in ranges:
        return []
    lo, hi = ranges[size_category.lower()]
    return [HardConstraint(ConstraintType.PIECES_MIN, lo, description=f"{size_category.title()} size minimum"),
            HardConstraint(ConstraintType.PIECES_MAX, hi, description=f"{size_category.title()} size maximum")]
