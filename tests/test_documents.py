"""Embedding-index documents: prep_vectorDB's row order and
_create_set_description / _estimate_complexity (lego_nlp_recommeder.py:196-267, 372-427),
restated in brickrec/documents.py, recorded beside the rows in the index file.

Parity UNPINNED: lego_nlp_recommeder.py does not import here (langchain / sentence-
transformers absent), so no golden output of the reference exists.  The expected
strings below are written out by hand from the reference's f-strings (:382-408)."""
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
