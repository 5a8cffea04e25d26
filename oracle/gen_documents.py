"""Golden a10 documents from the REFERENCE's own code — TEST INFRASTRUCTURE, build container only.

``lego_nlp_recommeder.py`` does not import here (langchain / sentence-transformers / torch-hub
loaders are absent), but the three pieces of it that build the embedding
documents are plain Python over a pandas row:

  * ``NLPRecommender._create_set_description``  (lego_nlp_recommeder.py:372-411)
  * ``NLPRecommender._estimate_complexity``     (:413-427)
  * the document loop of ``prep_vectorDB``       (:240-256: description + metadata per row)

plus the document SQL itself (:206-227).  This script reads the module's source as text,
takes those nodes out of its syntax tree (``ast``; nothing of the module is imported, none of
its other code runs), and executes them on a synthetic Rebrickable-shaped catalogue in sqlite:

  * the reference's SQL string, with the one Postgres-only aggregate rewritten for sqlite
    (``STRING_AGG(DISTINCT cat.name, ', ')`` -> a registered aggregate that joins the distinct
    names in ascending order, the order Postgres' sort-based DISTINCT produces);
  * ``pd.read_sql_query`` and ``df.iterrows()`` exactly as prep_vectorDB does;
  * ``Document`` replaced by a two-field record (langchain's class only stores the two).

Output: ``tests/golden/g6_documents.json`` — the query rows (inputs) and, per row in the
reference's order, the description, the metadata and the complexity label.  A sample of every
fifth row keeps the file small.  Usage: ``python oracle/gen_documents.py`` (needs
/root/reference; never run on the GPU box).
"""
from __future__ import annotations

import ast
import json
import os
import sqlite3
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.gen_golden import build_catalog  # noqa: E402

REF = "/root/reference/src/scripts/lego_nlp_recommeder.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "g6_documents.json")
CATEGORIES = ["Bricks", "Plates", "Tiles", "Minifig Accessories", "Technic Beams", "Windscreens", "Wheels and Tyres",
              "Bricks Sloped", "Plants and Animals", "Transportation - Sea and Air"]


def reference_nodes():
    """The two methods and prep_vectorDB's document loop, from the module's syntax tree."""
    tree = ast.parse(open(REF).read())
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "NLPRecommender")
    meth = {n.name: n for n in cls.body if isinstance(n, ast.FunctionDef)}
    prep = meth["prep_vectorDB"]
    sql = next(n.value.value for n in prep.body if isinstance(n, ast.Assign) and n.targets[0].id == "query")
    loop = [n for n in prep.body
            if (isinstance(n, ast.Assign) and getattr(n.targets[0], "id", "") == "docs")
            or (isinstance(n, ast.For) and isinstance(n.iter, ast.Call)
                and getattr(n.iter.func, "attr", "") == "iterrows")]
    assert len(loop) == 2, "prep_vectorDB's document loop not found"
    body = ast.Module(body=[ast.ClassDef(name="Ref", bases=[], keywords=[], decorator_list=[],
                                         body=[meth["_create_set_description"], meth["_estimate_complexity"]])]
                      + [ast.FunctionDef(name="build_docs", args=ast.arguments(
                          posonlyargs=[], args=[ast.arg("self"), ast.arg("df")], kwonlyargs=[], kw_defaults=[],
                          defaults=[]), body=loop + [ast.Return(ast.Name("docs", ast.Load()))], decorator_list=[])],
                      type_ignores=[])
    ast.fix_missing_locations(body)
    return compile(body, REF, "exec"), sql


class Document:
    """langchain_core.documents.Document's two fields."""

    def __init__(self, page_content, metadata):
        self.page_content, self.metadata = page_content, metadata


class StringAggDistinct:
    def __init__(self):
        self.v = set()

    def step(self, x):
        if x is not None:
            self.v.add(x)

    def finalize(self):
        return ", ".join(sorted(self.v)) if self.v else None


def catalogue_db():
    themes, sets, invs, iparts = build_catalog()
    rng = np.random.default_rng(23)
    db = sqlite3.connect(":memory:")
    c = db.cursor()
    c.execute("CREATE TABLE themes (id INTEGER PRIMARY KEY, name TEXT, parent_id INTEGER)")
    c.execute("CREATE TABLE sets (set_num TEXT PRIMARY KEY, name TEXT, year INTEGER, theme_id INTEGER,"
              " num_parts INTEGER, img_url TEXT)")
    c.execute("CREATE TABLE inventories (id INTEGER PRIMARY KEY, version INTEGER, set_num TEXT)")
    c.execute("CREATE TABLE inventory_parts (inventory_id INTEGER, part_num TEXT, color_id INTEGER,"
              " quantity INTEGER, is_spare INTEGER)")
    c.execute("CREATE TABLE inventory_minifigs (inventory_id INTEGER, fig_num TEXT, quantity INTEGER)")
    c.execute("CREATE TABLE parts (part_num TEXT PRIMARY KEY, name TEXT, part_cat_id INTEGER)")
    c.execute("CREATE TABLE part_categories (id INTEGER PRIMARY KEY, name TEXT)")
    c.executemany("INSERT INTO themes VALUES (?,?,?)", themes)
    c.executemany("INSERT INTO sets VALUES (?,?,?,?,?,?)", sets)
    c.executemany("INSERT INTO inventories VALUES (?,?,?)", invs)
    c.executemany("INSERT INTO inventory_parts VALUES (?,?,?,?,?)", iparts)
    c.executemany("INSERT INTO part_categories VALUES (?,?)", list(enumerate(CATEGORIES, 1)))
    # most parts have a category; a few reference a category id that does not exist (NULL name)
    c.executemany("INSERT INTO parts VALUES (?,?,?)",
                  [(f"p{i}", f"part {i}", int(rng.integers(1, len(CATEGORIES) + 3))) for i in range(4000)])
    figs = []
    for inv_id, _, _ in invs:
        for _ in range(int(rng.choice([0, 0, 0, 1, 2, 5]))):
            figs.append((inv_id, f"fig-{int(rng.integers(0, 3000)):06d}", 1))
    c.executemany("INSERT INTO inventory_minifigs VALUES (?,?,?)", figs)
    db.commit()
    db.create_aggregate("STRING_AGG_DISTINCT", 1, StringAggDistinct)
    return db


def main():
    code, sql = reference_nodes()
    pg_agg = "STRING_AGG(DISTINCT cat.name, ', ')"
    assert pg_agg in sql
    q = sql.replace(pg_agg, "STRING_AGG_DISTINCT(cat.name)")
    ns = {"pd": pd, "np": np, "Document": Document}
    exec(code, ns)
    db = catalogue_db()
    df = pd.read_sql_query(q, db)           # prep_vectorDB :233 (the reference's ORDER BY)
    docs = ns["build_docs"](ns["Ref"](), df)
    assert len(docs) == len(df)
    keep = list(range(0, len(df), 5))
    rows = df.iloc[keep].to_dict("records")
    out = {
        "source": "lego_nlp_recommeder.py:206-227 (SQL), :240-256 (document loop), :372-427 (description, "
                  "complexity) executed by oracle/gen_documents.py on a synthetic sqlite catalogue",
        "n_rows_total": int(len(df)),
        "rows": [{k: (None if (isinstance(v, float) and np.isnan(v)) else (int(v) if isinstance(v, (np.integer,)) else v))
                  for k, v in r.items()} for r in rows],
        "descriptions": [docs[i].page_content for i in keep],
        "metadata": [{k: (int(v) if isinstance(v, np.integer) else v) for k, v in docs[i].metadata.items()}
                     for i in keep],
    }
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0)
    print(f"{OUT}: {len(keep)} of {len(df)} documents")


if __name__ == "__main__":
    main()
