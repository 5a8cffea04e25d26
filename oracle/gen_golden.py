"""Generate golden fixtures from the REFERENCE itself — TEST INFRASTRUCTURE, build container only.

Runs the reference's own ``src/scripts/recommendation_system.py`` and
``src/scripts/hard_constraint_filter.py`` (imported from /root/reference, never copied)
against an in-memory sqlite catalogue, with ``psycopg2`` stubbed and a connection wrapper
that rewrites Postgres ``%s`` / ``= ANY(%s)`` placeholders for sqlite.
Outputs only data — inputs and the reference's outputs — into ``tests/golden/``:

  g1_content.npz     F=10 feat_matrix (as the reference built it) + similar-sets top-50,
                     with and without a valid-set filter (reference get_similar_sets)
  g2_semantic.npz    384-d fp32 unit vectors: similar-sets through the reference
                     (feat_matrix swapped for embeddings) and batched cosine queries through
                     sklearn.cosine_similarity, the function the reference calls (:214)
  g3_cf.npz          TruncatedSVD factors + CF top-2k lists for several users (reference)
  g4_hybrid.npz      constraint masks (reference apply_constraints over sqlite) and hybrid
                     final lists (reference HybridRecommender.get_recommendations)
  g5_faiss.npz       the reference's real MiniLM vectors (test_embeddings/index.faiss,
                     10x384) + their neighbour lists (reference get_similar_sets)
  catalog.json       the synthetic catalogue's string columns / theme names / reasons

Usage:  python oracle/gen_golden.py      (needs /root/reference; never run on the GPU box)
"""
from __future__ import annotations

import hashlib
import json
import os
import pickletools
import re
import sqlite3
import sys
import types
from datetime import datetime

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.restatement import unit_rows  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


# ----------------------------------------------------------------------------------------
# psycopg2 stub + sqlite connection wrapper
# ----------------------------------------------------------------------------------------
def install_psycopg2_stub():
    pg = types.ModuleType("psycopg2")
    extras = types.ModuleType("psycopg2.extras")
    extensions = types.ModuleType("psycopg2.extensions")

    class RealDictCursor:  # sentinel: the wrapper returns dict rows when asked for it
        pass

    extras.RealDictCursor = RealDictCursor
    extras.execute_values = lambda *a, **k: None
    extensions.connection = object

    def _connect(*a, **k):
        raise RuntimeError("psycopg2 stub: no Postgres in the build container")

    pg.connect = _connect
    pg.extras = extras
    pg.extensions = extensions
    pg.Error = Exception
    sys.modules["psycopg2"] = pg
    sys.modules["psycopg2.extras"] = extras
    sys.modules["psycopg2.extensions"] = extensions
    return RealDictCursor


_ANY = re.compile(r"=\s*ANY\(%s\)")


class _Cursor:
    def __init__(self, cur, as_dict):
        self._cur = cur
        self._dict = as_dict

    def execute(self, sql, params=None):
        params = list(params or [])
        out_sql, out_params, pi = [], [], 0
        for tok in re.split(r"(=\s*ANY\(%s\)|%s)", sql):
            if tok == "%s":
                out_sql.append("?")
                out_params.append(params[pi])
                pi += 1
            elif tok and _ANY.fullmatch(tok):
                val = list(params[pi])
                pi += 1
                out_sql.append("IN (" + ",".join("?" * len(val)) + ")")
                out_params.extend(val)
            else:
                out_sql.append(tok)
        self._cur.execute("".join(out_sql), out_params)
        return self

    @property
    def description(self):
        return self._cur.description

    def fetchall(self):
        rows = self._cur.fetchall()
        if self._dict:
            cols = [d[0] for d in self._cur.description]
            return [dict(zip(cols, r)) for r in rows]
        return rows

    def fetchone(self):
        r = self._cur.fetchone()
        if r is not None and self._dict:
            cols = [d[0] for d in self._cur.description]
            return dict(zip(cols, r))
        return r

    def close(self):
        self._cur.close()


class PgOnSqlite:
    def __init__(self, db, dict_factory):
        self._db = db
        self._dict_factory = dict_factory

    def cursor(self, cursor_factory=None):
        return _Cursor(self._db.cursor(), cursor_factory is self._dict_factory)

    def commit(self):
        self._db.commit()

    def rollback(self):
        self._db.rollback()

    def close(self):
        pass


# ----------------------------------------------------------------------------------------
# synthetic catalogue (Rebrickable-shaped)
# ----------------------------------------------------------------------------------------
THEMES = ["Star Wars", "Star Wars Episode IV", "City", "City Police", "Technic", "Creator",
          "Creator Expert", "Ninjago", "Friends", "Harry Potter", "Ideas", "Architecture",
          "Duplo", "Speed Champions", "Marvel Super Heroes", "Classic Space", "Space",
          "Castle", "Pirates", "Train", "Minecraft", "Jurassic World", "Disney",
          "Botanical Collection", "Art", "Icons", "Modular Buildings", "Bionicle",
          "Hidden Side", "Monkie Kid"]


def build_catalog(n_sets=2000, seed=7):
    rng = np.random.default_rng(seed)
    themes = [(i + 1, name, (1 if name.startswith("Star Wars ") else
                             3 if name.startswith("City ") else None))
              for i, name in enumerate(THEMES)]
    set_nums = sorted({f"{int(v)}-1" for v in rng.choice(np.arange(1000, 99999), n_sets, replace=False)})
    sets, invs, iparts = [], [], []
    inv_id = 1
    for s in set_nums:
        parts = int(np.exp(rng.uniform(np.log(5), np.log(7000))))
        if rng.random() < 0.03:
            parts = 0  # accessories / catalogues: excluded by num_parts > 0
        year = int(rng.integers(1975, 2026))
        theme = int(rng.integers(1, len(THEMES) + 1))
        sets.append((s, f"Set {s} {THEMES[theme - 1]}", year, theme, parts, f"https://img/{s}.jpg"))
        invs.append((inv_id, 1, s))
        n_uniq = int(max(1, min(parts, rng.integers(1, 60)))) if parts > 0 else int(rng.integers(0, 3))
        n_col = int(rng.integers(1, 25))
        used = set()
        for j in range(n_uniq):
            part_num = f"p{int(rng.integers(0, 4000))}"
            color = int(rng.integers(0, n_col))
            spare = bool(rng.random() < 0.1)
            key = (part_num, color, spare)
            if key in used:
                continue
            used.add(key)
            iparts.append((inv_id, part_num, color, int(rng.integers(1, 40)), int(spare)))
        inv_id += 1
    return themes, sets, invs, iparts


def make_db(themes, sets, invs, iparts, owned=(), wished=()):
    db = sqlite3.connect(":memory:")
    c = db.cursor()
    c.execute("CREATE TABLE themes (id INTEGER PRIMARY KEY, name TEXT, parent_id INTEGER)")
    c.execute("CREATE TABLE sets (set_num TEXT PRIMARY KEY, name TEXT, year INTEGER, theme_id INTEGER,"
              " num_parts INTEGER, img_url TEXT)")
    c.execute("CREATE TABLE inventories (id INTEGER PRIMARY KEY, version INTEGER, set_num TEXT)")
    c.execute("CREATE TABLE inventory_parts (inventory_id INTEGER, part_num TEXT, color_id INTEGER,"
              " quantity INTEGER, is_spare INTEGER)")
    c.execute("CREATE TABLE user_interactions (id INTEGER PRIMARY KEY, user_id INTEGER, set_num TEXT,"
              " interaction_type TEXT, rating INTEGER, created_at TEXT)")
    c.execute("CREATE TABLE user_collections (id INTEGER PRIMARY KEY, user_id INTEGER, set_num TEXT)")
    c.execute("CREATE TABLE user_wishlists (id INTEGER PRIMARY KEY, user_id INTEGER, set_num TEXT)")
    c.executemany("INSERT INTO themes VALUES (?,?,?)", themes)
    c.executemany("INSERT INTO sets VALUES (?,?,?,?,?,?)", sets)
    c.executemany("INSERT INTO inventories VALUES (?,?,?)", invs)
    c.executemany("INSERT INTO inventory_parts VALUES (?,?,?,?,?)", iparts)
    c.executemany("INSERT INTO user_collections (user_id, set_num) VALUES (?,?)", owned)
    c.executemany("INSERT INTO user_wishlists (user_id, set_num) VALUES (?,?)", wished)
    db.commit()
    return db


# ----------------------------------------------------------------------------------------
def min_gap(scores, k):
    s = np.sort(np.asarray(scores, np.float64))[::-1][: k + 1]
    return float(np.min(s[:-1] - s[1:])) if len(s) > 1 else 1.0


def recs_to_arrays(recs, index_of):
    ids = np.array([index_of[r.set_num] for r in recs], dtype=np.int64)
    sc = np.array([r.score for r in recs], dtype=np.float64)
    return ids, sc


def read_faiss_flat(path):
    """``IxF2`` (IndexFlatL2) file: header, then ntotal*d float32 — read as raw bytes."""
    b = open(path, "rb").read()
    assert b[:4] == b"IxF2"
    d = int(np.frombuffer(b, np.int32, 1, 4)[0])
    ntotal = int(np.frombuffer(b, np.int64, 1, 8)[0])
    off = len(b) - ntotal * d * 4
    x = np.frombuffer(b, np.float32, ntotal * d, off).reshape(ntotal, d).copy()
    return x, off


def faiss_docstore_set_nums(path):
    """Set numbers in row order from ``index.pkl`` by parsing its opcode stream with
    ``pickletools.genops`` — nothing in the file is unpickled or executed."""
    out, want, memo, last = [], False, {}, None
    for op, arg, _ in pickletools.genops(open(path, "rb").read()):
        if op.name == "MEMOIZE":
            memo[len(memo)] = last
            continue
        val = memo.get(arg) if op.name in ("BINGET", "LONG_BINGET") else arg
        last = val if isinstance(val, str) else None
        if isinstance(val, str):
            if want:
                out.append(val)
                want = False
            elif val == "set_num":
                want = True
    return out


def main():
    rdc = install_psycopg2_stub()
    sys.path.insert(0, os.path.join(REF, "src", "scripts"))
    import recommendation_system as rs      # noqa: E402  (the reference itself)
    import hard_constraint_filter as hcf    # noqa: E402

    os.makedirs(OUT, exist_ok=True)
    themes, sets, invs, iparts = build_catalog()
    set_index = {s[0]: i for i, s in enumerate(s for s in sets)}
    # owned / wishlisted sets for two users (exclude_owned / exclude_wishlisted)
    rng = np.random.default_rng(11)
    owned = [(3, sets[int(i)][0]) for i in rng.choice(len(sets), 60, replace=False)]
    wished = [(3, sets[int(i)][0]) for i in rng.choice(len(sets), 40, replace=False)]
    db = make_db(themes, sets, invs, iparts, owned, wished)
    conn = PgOnSqlite(db, rdc)

    # ---------------- G1: content path --------------------------------------------------
    cb = rs.ContentBasedRecommender(conn)
    cb.prepare_features()
    feat = np.asarray(cb.feat_matrix, dtype=np.float64)
    sf = cb.set_feat
    row_set = list(sf["set_num"])            # content item space: sets with num_parts>0, by set_num
    n1 = len(row_set)
    # valid filter: pieces <= 800 and year >= 2005 (restated predicate; checked in G4 too)
    filt = [s for s, p, y in zip(sf["set_num"], sf["num_parts"], sf["year"]) if p <= 800 and y >= 2005]
    k1 = 50
    cand = list(range(0, n1, 7))
    qrows, res_nf, res_f, reasons_nf = [], [], [], []
    for qi in cand:
        recs = cb.get_similar_sets(row_set[qi], k1)
        recs_f = cb.get_similar_sets(row_set[qi], k1, valid_set_filter=filt)
        idx_of = {s: i for i, s in enumerate(row_set)}
        a_i, a_s = recs_to_arrays(recs, idx_of)
        b_i, b_s = recs_to_arrays(recs_f, idx_of)
        # keep queries whose rankings are unambiguous at fp32 precision
        sim = np.asarray(__import__("sklearn.metrics.pairwise", fromlist=["x"]).cosine_similarity(
            feat[qi:qi + 1], feat))[0]
        top = np.sort(sim)[::-1][: k1 + 3]
        if np.min(top[:-1] - top[1:]) < 2e-6:
            continue
        allowed = np.array([s in set(filt) for s in row_set])
        st = np.sort(sim[allowed])[::-1][: k1 + 3]
        if len(st) > 1 and np.min(st[:-1] - st[1:]) < 2e-6:
            continue
        qrows.append(qi)
        res_nf.append((a_i, a_s))
        res_f.append((b_i, b_s))
        reasons_nf.append([list(r.reasons) for r in recs])
        if len(qrows) == 16:
            break
    assert len(qrows) >= 8, f"only {len(qrows)} unambiguous content queries"
    np.savez_compressed(
        os.path.join(OUT, "g1_content.npz"),
        feat_matrix=feat, query_rows=np.array(qrows, np.int64), k=np.int64(k1),
        filter_mask=np.array([s in set(filt) for s in row_set]),
        ids_nofilter=np.stack([r[0] for r in res_nf]), scores_nofilter=np.stack([r[1] for r in res_nf]),
        ids_filter=np.stack([r[0] for r in res_f]), scores_filter=np.stack([r[1] for r in res_f]),
        num_parts=np.asarray(sf["num_parts"], np.int64), year=np.asarray(sf["year"], np.int64),
        theme_id=np.asarray(sf["theme_id"], np.int64),
        complexity_score=np.asarray(sf["complexity_score"], np.float64),
    )
    catalog = {
        "row_set_nums": row_set,
        "names": list(sf["name"]),
        "theme_names": [t if isinstance(t, str) else None for t in sf["theme_name"]],
        "img_urls": list(sf["img_url"]),
        "size_category": list(sf["size_category"]),
        "themes": {str(t[0]): t[1] for t in themes},
        "g1_reasons_nofilter": reasons_nf,
        "generated_year": datetime.now().year,
    }

    # ---------------- G3: collaborative filtering ----------------------------------------
    cf = rs.CollaborativeFilteringRecommender(conn)
    cf.prepare_user_item_matrix()
    cf.train_svd_model()
    cols = list(cf.user_item_matrix.columns)
    users = [1, 2, 7, 19, 42, 50]
    k3 = 10
    cf_ids, cf_scores, cf_len = [], [], []
    for u in users:
        recs = cf.get_recommendations(u, 2 * k3)
        ids, sc = recs_to_arrays(recs, {s: i for i, s in enumerate(cols)})
        cf_len.append(len(ids))
        cf_ids.append(np.pad(ids, (0, 2 * k3 - len(ids)), constant_values=-1))
        cf_scores.append(np.pad(sc, (0, 2 * k3 - len(sc))))
    # unknown user (the API passes str(user_id)): the reference falls back to cold start
    cold = cf.get_recommendations("5", k3)
    np.savez_compressed(
        os.path.join(OUT, "g3_cf.npz"),
        user_factors=np.asarray(cf.user_factors, np.float64),
        item_factors=np.asarray(cf.item_factors, np.float64),
        rated=np.asarray(cf.user_item_matrix.values > 0),
        user_ids=np.asarray(cf.user_item_matrix.index, np.int64),
        query_users=np.array(users, np.int64), k=np.int64(k3),
        ids=np.stack(cf_ids), scores=np.stack(cf_scores), lens=np.array(cf_len, np.int64),
        cold_start_len=np.int64(len(cold)),
    )
    catalog["cf_columns"] = cols

    # ---------------- G4: hard-constraint masks + hybrid ---------------------------------
    hy = rs.HybridRecommender(conn)
    hy.content_recommender = cb
    hy.collaborative_recommender = cf
    cases = [
        dict(pieces_max=800, year_min=2005),
        dict(price_max=45.0),
        dict(price_min=20.0, max_complexity="moderate"),
        dict(age_min=6, required_themes=["star wars"]),
        dict(age_min=14, excluded_themes=["City", "Duplo"]),
        dict(age_max=10, min_complexity="moderate"),
        dict(must_be_available=True),
        dict(exclude_owned=True, exclude_wishlisted=True, user_id=3),
        dict(required_themes=["no-such-theme"]),
        dict(pieces_min=100, pieces_max=3000, year_max=2020, excluded_themes=["technic"]),
    ]
    masks = []
    for cs in cases:
        cons = hy.constraint_filter.create_constraint_set(**cs)
        res = hy.constraint_filter.apply_constraints(cons)
        vs = set(res.valid_set_nums)
        masks.append(np.array([s in vs for s in row_set]))
    # hybrid: (user, liked_set, constraint case)
    cf_rows = {s: i for i, s in enumerate(row_set)}
    hcases = [(1, 0, 0), (2, 3, 1), (7, 5, None), (19, 9, 2), (42, 2, 4), (50, 11, 9), (None, 4, 0), (3, None, 0)]
    k4 = 10
    h_ids, h_sc, h_len, h_meta = [], [], [], []
    for (u, qpos, ci) in hcases:
        liked = row_set[qrows[qpos]] if qpos is not None else None
        cons = hy.constraint_filter.create_constraint_set(**cases[ci]) if ci is not None else None
        recs, _ = hy.get_recommendations(user_id=u, liked_set=liked, top_k=k4, constraints=cons)
        ids = np.array([cf_rows[r.set_num] for r in recs], np.int64)
        sc = np.array([r.score for r in recs], np.float64)
        h_len.append(len(ids))
        h_ids.append(np.pad(ids, (0, k4 - len(ids)), constant_values=-1))
        h_sc.append(np.pad(sc, (0, k4 - len(sc))))
        h_meta.append((-1 if u is None else u, -1 if qpos is None else qrows[qpos], -1 if ci is None else ci))
    np.savez_compressed(
        os.path.join(OUT, "g4_hybrid.npz"),
        masks=np.stack(masks), case_json=np.array([json.dumps(c) for c in cases]),
        hybrid_meta=np.array(h_meta, np.int64), k=np.int64(k4),
        ids=np.stack(h_ids), scores=np.stack(h_sc), lens=np.array(h_len, np.int64),
        owned_rows=np.array([cf_rows[s] for u, s in owned if s in cf_rows], np.int64),
        wished_rows=np.array([cf_rows[s] for u, s in wished if s in cf_rows], np.int64),
        current_year=np.int64(datetime.now().year),
    )

    # ---------------- G2: 384-d fp32 unit vectors ---------------------------------------
    from sklearn.metrics.pairwise import cosine_similarity
    n2, d2, b2, k2 = 4096, 384, 16, 50
    x = unit_rows(n2, d2, 1234)          # regenerated bit-identically by the tests (sha256 kept)
    q = unit_rows(b2, d2, 4321)
    # (a) through the reference: get_similar_sets over an embedding matrix
    cb2 = rs.ContentBasedRecommender(conn)
    cb2.set_feat = pd.DataFrame({
        "set_num": [f"e{i}" for i in range(n2)], "name": [f"e{i}" for i in range(n2)],
        "theme_id": np.zeros(n2, np.int64), "theme_name": ["t"] * n2, "size_category": ["small"] * n2,
        "complexity_score": np.zeros(n2), "year": np.full(n2, 2020), "num_parts": np.full(n2, 10),
        "img_url": [None] * n2})
    cb2.feat_matrix = x
    sim_q = [int(v) for v in np.random.default_rng(99).choice(n2, b2, replace=False)]
    s_ids, s_sc = [], []
    for qi in sim_q:
        recs = cb2.get_similar_sets(f"e{qi}", k2)
        ids, sc = recs_to_arrays(recs, {f"e{i}": i for i in range(n2)})
        s_ids.append(ids)
        s_sc.append(sc)
    # (b) batched semantic queries: cosine_similarity (the call at :214) + argsort desc
    sim = cosine_similarity(q, x)
    order = np.argsort(sim, axis=1)[:, ::-1][:, :k2]
    gaps = [min_gap(sim[i], k2) for i in range(b2)]
    np.savez_compressed(
        os.path.join(OUT, "g2_semantic.npz"), items_sha256=np.array(hashlib.sha256(x.tobytes()).hexdigest()),
        n_items=np.int64(n2), queries=q, k=np.int64(k2),
        similar_rows=np.array(sim_q, np.int64), similar_ids=np.stack(s_ids), similar_scores=np.stack(s_sc),
        semantic_ids=order.astype(np.int64), semantic_scores=np.take_along_axis(sim, order, 1),
        min_gap=np.array(gaps))

    # ---------------- G5: the reference's real MiniLM vectors ---------------------------
    xf, off = read_faiss_flat(os.path.join(REF, "test_embeddings", "index.faiss"))
    fnums = faiss_docstore_set_nums(os.path.join(REF, "test_embeddings", "index.pkl"))
    assert len(fnums) == xf.shape[0]
    cb5 = rs.ContentBasedRecommender(conn)
    nf = xf.shape[0]
    cb5.set_feat = pd.DataFrame({
        "set_num": fnums, "name": fnums, "theme_id": np.zeros(nf, np.int64), "theme_name": ["t"] * nf,
        "size_category": ["xl"] * nf, "complexity_score": np.zeros(nf), "year": np.full(nf, 2020),
        "num_parts": np.full(nf, 10), "img_url": [None] * nf})
    cb5.feat_matrix = xf
    f_ids, f_sc = [], []
    for s in fnums:
        recs = cb5.get_similar_sets(s, nf - 1)
        ids, sc = recs_to_arrays(recs, {t: i for i, t in enumerate(fnums)})
        f_ids.append(ids)
        f_sc.append(sc)
    np.savez_compressed(
        os.path.join(OUT, "g5_faiss.npz"), vectors=xf, header_offset=np.int64(off),
        set_nums=np.array(fnums), ids=np.stack(f_ids), scores=np.stack(f_sc))

    with open(os.path.join(OUT, "catalog.json"), "w") as f:
        json.dump(catalog, f)
    print("golden fixtures written:", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
