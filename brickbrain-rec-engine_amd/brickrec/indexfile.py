"""Item-index file: the embedding matrix plus the catalogue columns the scoring path needs,
in one binary file that is memory-mapped, not parsed.

The reference rebuilds its item matrix on every start: ``prep_vectorDB`` selects the sets
``ORDER BY num_parts DESC, year DESC`` and encodes one document per set into pgvector
(lego_nlp_recommeder.py:196-267), and ``_create_feature_matrix`` rebuilds the content
features (recommendation_system.py:175-192).  Here whichever matrix was built (MiniLM
embeddings, content features, or synthetic rows) is written once, and a server maps the
file and uploads it to HBM: the rows go from page cache to the device in the library's
staging chunks, with no Python-side copy.

Layout (little endian; every section 4-KiB aligned)::

    0   magic "BBIX", u32 version (2; 1 is read too), u64 n, u32 d, u32 flags (bit 0: rows
        unit-norm, bit 1: attributes, bit 2: documents), u64 off_rows, u64 off_attrs,
        u64 off_names, u64 names_bytes, [v2] u64 off_docs, u64 docs_bytes
    off_rows   f32 [n][d]                      item rows (row i = global id i)
    off_attrs  i32 num_parts[n], i16 year[n], i32 theme_id[n]   (bb_upload_attrs columns)
    off_names  UTF-8 JSON list of set_num strings (row order)
    off_docs   UTF-8 JSON {"descriptions": [n], "metadata": [n]} — the document each row
               embeds (brickrec/documents.py: prep_vectorDB's text, in its row order)

Data only: nothing in the file is executed, and readers check every offset against the
file size.
"""
from __future__ import annotations

import json
import os
import struct
from typing import List, Optional, Sequence

import numpy as np

MAGIC = b"BBIX"
VERSION = 2
_HDR = struct.Struct("<4sIQIIQQQQ")     # v1 header
_HDR2 = struct.Struct("<QQ")            # v2 extension: off_docs, docs_bytes
_ALIGN = 4096


def _align(x: int) -> int:
    return (x + _ALIGN - 1) // _ALIGN * _ALIGN


def write_index(path: str, set_nums: Sequence[str], rows: np.ndarray, num_parts=None, year=None, theme_id=None,
                unit_norm: bool = False, documents=None) -> None:
    """Write rows (n×d, stored as f32), the optional attribute columns, and optionally the
    documents the rows embed: (descriptions, metadata) lists in row order, e.g. from
    documents.build_documents."""
    rows = np.asarray(rows)
    n, d = rows.shape
    if len(set_nums) != n:
        raise ValueError("one set_num per row")
    names = json.dumps([str(s) for s in set_nums]).encode()
    docs = b""
    if documents is not None:
        desc, meta = documents
        if len(desc) != n or len(meta) != n:
            raise ValueError("one document per row")
        docs = json.dumps({"descriptions": list(desc), "metadata": list(meta)}).encode()
    off_rows = _align(_HDR.size + _HDR2.size)
    off_attrs = _align(off_rows + n * d * 4)
    has_attrs = num_parts is not None
    off_names = _align(off_attrs + (n * 10 if has_attrs else 0))
    off_docs = _align(off_names + len(names))
    flags = (1 if unit_norm else 0) | (2 if has_attrs else 0) | (4 if docs else 0)
    with open(path, "wb") as f:
        f.write(_HDR.pack(MAGIC, VERSION, n, d, flags, off_rows, off_attrs, off_names, len(names)))
        f.write(_HDR2.pack(off_docs if docs else 0, len(docs)))
        f.seek(off_rows)
        for i in range(0, n, 1 << 16):  # bounded host memory for large matrices
            f.write(np.ascontiguousarray(rows[i:i + (1 << 16)], dtype=np.float32).tobytes())
        if has_attrs:
            f.seek(off_attrs)
            f.write(np.ascontiguousarray(num_parts, np.int32).tobytes())
            f.write(np.ascontiguousarray(np.clip(year, -32768, 32767), np.int16).tobytes())
            f.write(np.ascontiguousarray(theme_id, np.int32).tobytes())
        f.seek(off_names)
        f.write(names)
        if docs:
            f.seek(off_docs)
            f.write(docs)


class IndexFile:
    """A mapped index file: ``rows`` (np.memmap f32 n×d), ``set_nums``, and the attribute
    columns (or None)."""

    def __init__(self, path: str):
        size = os.path.getsize(path)
        with open(path, "rb") as f:
            hdr = f.read(_HDR.size + _HDR2.size)
        if len(hdr) < _HDR.size:
            raise ValueError(f"{path}: truncated header")
        magic, ver, n, d, flags, off_rows, off_attrs, off_names, names_bytes = _HDR.unpack(hdr[:_HDR.size])
        if magic != MAGIC or ver not in (1, 2):
            raise ValueError(f"{path}: not a brickrec index file (v1 / v2)")
        off_docs = docs_bytes = 0
        if ver >= 2:
            if len(hdr) < _HDR.size + _HDR2.size:
                raise ValueError(f"{path}: truncated header")
            off_docs, docs_bytes = _HDR2.unpack(hdr[_HDR.size:])
        has_attrs = bool(flags & 2)
        if (off_rows + n * d * 4 > size or (has_attrs and off_attrs + n * 10 > size)
                or off_names + names_bytes > size or (flags & 4 and off_docs + docs_bytes > size)):
            raise ValueError(f"{path}: sections past the end of the file")
        self.path, self.n, self.d = path, int(n), int(d)
        self.unit_norm = bool(flags & 1)
        self.rows = np.memmap(path, np.float32, "r", off_rows, (self.n, self.d))
        if has_attrs:
            self.num_parts = np.memmap(path, np.int32, "r", off_attrs, (self.n,))
            self.year = np.memmap(path, np.int16, "r", off_attrs + 4 * self.n, (self.n,))
            self.theme_id = np.memmap(path, np.int32, "r", off_attrs + 6 * self.n, (self.n,))
        else:
            self.num_parts = self.year = self.theme_id = None
        with open(path, "rb") as f:
            f.seek(off_names)
            self.set_nums: List[str] = json.loads(f.read(names_bytes).decode())
        if len(self.set_nums) != self.n:
            raise ValueError(f"{path}: {len(self.set_nums)} names for {self.n} rows")
        self.descriptions = self.metadata = None
        if flags & 4:
            with open(path, "rb") as f:
                f.seek(off_docs)
                dd = json.loads(f.read(docs_bytes).decode())
            self.descriptions, self.metadata = dd["descriptions"], dd["metadata"]
            if len(self.descriptions) != self.n or len(self.metadata) != self.n:
                raise ValueError(f"{path}: document count does not match the rows")

    def load_into(self, index, present: Optional[np.ndarray] = None):
        """Upload the rows (and attributes) into an ``ItemIndex`` straight from the mapping."""
        index.upload_items(self.rows, prenormalized=self.unit_norm, present=present)
        if self.num_parts is not None:
            index.upload_attrs(self.num_parts, self.year, self.theme_id)
        return index


def open_index(path: str) -> IndexFile:
    return IndexFile(path)
