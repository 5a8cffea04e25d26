"""Embedding-index documents: prep_vectorDB's row order and
_create_set_description / _estimate_complexity (lego_nlp_recommeder.py:196-267, 372-427),
restated in brickrec/documents.py, recorded beside the rows in the index file.

Parity PINNED (round 5): tests/golden/g6_documents.json holds what the reference's own code
produced — oracle/gen_documents.py takes _create_set_description, _estimate_complexity and
prep_vectorDB's document loop out of the module's syntax tree (the module itself does not
import: langchain / sentence-transformers are absent) and runs them, with the
reference's document SQL, on a synthetic sqlite catalogue.  The hand-written cases below keep
the NULL-count edge (a NaN colour count), which Postgres' COUNT never produces."""
import json
import os

import numpy as np

from brickrec.documents import build_documents, create_set_description, estimate_complexity, order_rows

ROWS = [
    {"set_num": "10294-1", "name": "Titanic", "year": 2021, "num_parts": 9090, "theme_name": "Icons",
     "parent_theme_name": None, "num_colors": 34, "num_minifigs": 0, "part_categories": "Bricks, Plates"},
    {"set_num": "75192-1", "name": "Millennium Falcon", "year": 2017, "num_parts": 7541, "theme_name": "Ultimate Collector Series",
     "parent_theme_name": "Star Wars", "num_colors": 18, "num_minifigs": 8, "part_categories": None},
    {"set_num": "30000-1", "name": "Tiny", "year": 2010, "num_parts": 40, "theme_name": "City",
     "parent_theme_name": "City", "num_colors": 3, "num_minifigs": 1, "part_categories": ""},
    {"set_num": "40000-1", "name": "Mid", "year": 2012, "num_parts": 500, "theme_name": "Castle",
     "parent_theme_name": None, "num_colors": 10, "num_minifigs": 2, "part_categories": "Minifig Accessories"},
    {"set_num": "40001-1", "name": "Mid2", "year": 2015, "num_parts": 500, "theme_name": "Castle",
     "parent_theme_name": None, "num_colors": float("nan"), "num_minifigs": 0, "part_categories": None},
    {"set_num": "0-1", "name": "Empty", "year": 2000, "num_parts": 0, "theme_name": "x",
     "parent_theme_name": None, "num_colors": 0, "num_minifigs": 0, "part_categories": None},
]


def test_descriptions_and_complexity():
    assert create_set_description(ROWS[0]) == (
        "LEGO Titanic (Set 10294-1). from the Icons theme. released in 2021. with 9090 pieces. "
        "featuring 34 different colors. contains parts from categories: Bricks, Plates. "
        "challenging build for experienced builders")
    assert create_set_description(ROWS[1]) == (
        "LEGO Millennium Falcon (Set 75192-1). from the Ultimate Collector Series theme. part of the Star Wars "
        "collection. released in 2017. with 7541 pieces. featuring 18 different colors. includes 8 minifigures. "
        "challenging build for experienced builders")
    assert create_set_description(ROWS[2]) == (
        "LEGO Tiny (Set 30000-1). from the City theme. released in 2010. with 40 pieces. featuring 3 different "
        "colors. includes 1 minifigures. suitable for beginners with straightforward building")
    assert [estimate_complexity(r) for r in ROWS[:5]] == ["complex", "complex", "simple", "moderate", "simple"]


def test_row_order_and_index_file(tmp_path):
    from brickrec.indexfile import open_index, write_index
    ordered = order_rows(ROWS)
    # ORDER BY num_parts DESC, year DESC; num_parts > 0 only
    assert [r["set_num"] for r in ordered] == ["10294-1", "75192-1", "40001-1", "40000-1", "30000-1"]
    names, desc, meta = build_documents(ROWS)
    assert names == [r["set_num"] for r in ordered] and len(desc) == 5
    assert meta[2] == {"set_num": "40001-1", "name": "Mid2", "year": 2015, "num_parts": 500, "theme": "Castle",
                       "parent_theme": None, "num_colors": 0, "num_minifigs": 0, "complexity": "simple"}
    x = np.eye(5, 8, dtype=np.float32)
    p = str(tmp_path / "docs.bbix")
    write_index(p, names, x, documents=(desc, meta), unit_norm=True)
    f = open_index(p)
    assert f.set_nums == names and f.descriptions == desc and f.metadata == meta
    np.testing.assert_array_equal(np.asarray(f.rows), x)
    assert build_documents(ROWS, limit=2)[0] == ["10294-1", "75192-1"]


G6 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "g6_documents.json")


def test_documents_match_the_reference_golden():
    """Every sampled row of the reference's document query: the restated description, metadata
    and complexity equal what the reference's code produced from the same row."""
    from brickrec.documents import document_metadata
    g = json.load(open(G6))
    assert len(g["rows"]) == len(g["descriptions"]) == len(g["metadata"]) > 300
    for row, desc, meta in zip(g["rows"], g["descriptions"], g["metadata"]):
        assert create_set_description(row) == desc, row["set_num"]
        assert document_metadata(row) == meta, row["set_num"]
        assert estimate_complexity(row) == meta["complexity"]


def test_row_order_matches_the_reference_golden():
    """ORDER BY num_parts DESC, year DESC (the reference's SQL, run by the generator): the
    restated order of the same rows, given in any order, is the reference's up to rows tied
    on both keys (whose order the SQL leaves open)."""
    g = json.load(open(G6))
    rows = g["rows"]
    perm = np.random.default_rng(5).permutation(len(rows))
    ordered = order_rows([rows[i] for i in perm])
    key = lambda r: (r["num_parts"], r["year"])
    assert [key(r) for r in ordered] == [key(r) for r in rows]
    groups = {}
    for r in rows:
        groups.setdefault(key(r), set()).add(r["set_num"])
    for r in ordered:
        assert r["set_num"] in groups[key(r)]
