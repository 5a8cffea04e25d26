"""Embedding-index documents: the rows and texts ``NLPRecommender.prep_vectorDB`` encodes
(lego_nlp_recommeder.py:196-267, 372-427).

The reference selects every set with parts, aggregated with its themes, colours, minifigures
and part categories, ``ORDER BY s.num_parts DESC, s.year DESC`` (:205-227), builds one
description per row (``_create_set_description`` :372-410) and encodes it with MiniLM
(``normalize_embeddings=True``).  The encoder is out of scope (its weights are fetched by
name); this module restates the row order, the text and the metadata, so that an index
file (``indexfile.write_index(..., documents=...)``) records which document each embedding
row is and a later encoder run can be lined up with it.

Parity is pinned by ``tests/golden/g6_documents.json``: the module that holds these functions
does not import here (langchain and sentence-transformers are absent), so
``oracle/gen_documents.py`` runs the reference's own three pieces of code (taken out of its
syntax tree) and its SQL on a synthetic catalogue, and ``tests/test_documents.py`` compares
every sampled row.  Two choices the SQL leaves open are fixed here and documented: rows tied on
(num_parts, year) keep their input order (set_num ascending from ``document_rows``), and
``STRING_AGG(DISTINCT cat.name, ', ')`` lists the categories in ascending order (what
Postgres' sort-based DISTINCT produces).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

DOCUMENT_SQL = """
SELECT s.set_num, s.name, s.year, s.num_parts,
       t.name as theme_name, pt.name as parent_theme_name,
       COUNT(DISTINCT ip.color_id) as num_colors,
       COUNT(DISTINCT im.fig_num) as num_minifigs,
       STRING_AGG(DISTINCT cat.name, ', ') as part_categories
FROM sets s
LEFT JOIN themes t ON s.theme_id = t.id
LEFT JOIN themes pt ON t.parent_id = pt.id
LEFT JOIN inventories i ON s.set_num = i.set_num
LEFT JOIN inventory_parts ip ON i.id = ip.inventory_id
LEFT JOIN inventory_minifigs im ON i.id = im.inventory_id
LEFT JOIN parts p ON ip.part_num = p.part_num
LEFT JOIN part_categories cat ON p.part_cat_id = cat.id
WHERE s.num_parts > 0
GROUP BY s.set_num, s.name, s.year, s.num_parts, t.name, pt.name
ORDER BY s.num_parts DESC, s.year DESC
"""  # lego_nlp_recommeder.py:205-227 (Postgres; LIMIT appended by prep_vectorDB when asked)


def _isnan(v) -> bool:
    return isinstance(v, float) and math.isnan(v)


def estimate_complexity(row: Dict) -> str:
    """``_estimate_complexity`` (:412-427): < 100 parts or < 5 colours -> simple, > 1000 parts
    or > 20 colours -> complex, else moderate (a NULL colour count reads as 0)."""
    colors = row.get("num_colors")
    colors = 0 if colors is None or _isnan(colors) else colors
    if row["num_parts"] < 100 or colors < 5:
        return "simple"
    if row["num_parts"] > 1000 or colors > 20:
        return "complex"
    return "moderate"


def create_set_description(row: Dict) -> str:
    """``_create_set_description`` (:372-410): the sentence parts joined by ". "."""
    parts = [f"LEGO {row['name']} (Set {row['set_num']})", f"from the {row['theme_name']} theme"]
    parent = row.get("parent_theme_name")
    if parent and parent != row["theme_name"]:          # Python truthiness, as the reference
        parts.append(f"part of the {parent} collection")
    parts += [f"released in {row['year']}", f"with {row['num_parts']} pieces"]
    nc = row.get("num_colors")
    if nc is not None and not _isnan(nc) and nc > 0:
        parts.append(f"featuring {nc} different colors")
    nm = row.get("num_minifigs")
    if nm is not None and not _isnan(nm) and nm > 0:
        parts.append(f"includes {nm} minifigures")
    if row.get("part_categories"):
        parts.append(f"contains parts from categories: {row['part_categories']}")
    cx = estimate_complexity(row)
    if cx == "simple":
        parts.append("suitable for beginners with straightforward building")
    elif cx == "complex":
        parts.append("challenging build for experienced builders")
    else:
        parts.append("moderate complexity suitable for most builders")
    return ". ".join(parts)


def document_metadata(row: Dict) -> Dict:
    """The per-document metadata dict of prep_vectorDB (:243-253)."""
    nc, nm = row.get("num_colors"), row.get("num_minifigs")
    return {"set_num": row["set_num"], "name": row["name"], "year": int(row["year"]),
            "num_parts": int(row["num_parts"]), "theme": row["theme_name"],
            "parent_theme": row.get("parent_theme_name"),
            "num_colors": int(nc) if nc is not None and not _isnan(nc) else 0,
            "num_minifigs": int(nm) if nm is not None and not _isnan(nm) else 0,
            "complexity": estimate_complexity(row)}


def order_rows(rows: Sequence[Dict], limit: Optional[int] = None) -> List[Dict]:
    """``WHERE num_parts > 0 ... ORDER BY num_parts DESC, year DESC [LIMIT n]`` (:225-231);
    ties keep their input order."""
    kept = [r for r in rows if r["num_parts"] is not None and r["num_parts"] > 0]
    kept = sorted(kept, key=lambda r: (-r["num_parts"], -r["year"]))
    return kept[:limit] if limit else kept


def build_documents(rows: Sequence[Dict], limit: Optional[int] = None) -> Tuple[List[str], List[str], List[Dict]]:
    """Rows of the document query (any order) -> (set_nums, descriptions, metadata) in the
    embedding-row order of prep_vectorDB: row i of the encoded matrix is document i."""
    ordered = order_rows(rows, limit)
    return ([r["set_num"] for r in ordered], [create_set_description(r) for r in ordered],
            [document_metadata(r) for r in ordered])


def document_rows(dbcon, limit: Optional[int] = None) -> List[Dict]:
    """Run the document query on the reference's Postgres schema (set_num ascending first, so
    equal sort keys keep a fixed order)."""
    import pandas as pd
    q = DOCUMENT_SQL.replace("ORDER BY s.num_parts DESC, s.year DESC",
                             "ORDER BY s.num_parts DESC, s.year DESC, s.set_num ASC")
    if limit:
        q += f" LIMIT {int(limit)}"
    return pd.read_sql_query(q, dbcon).to_dict("records")
