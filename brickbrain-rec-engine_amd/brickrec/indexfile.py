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

    0   magic "BBIX", u32 version (1), u64 n, u32 d, u32 flags (bit 0: rows unit-norm),
        u64 off_rows, u64 off_attrs, u64 off_names, u64 names_bytes
    off_rows   f32 [n][d]                      item rows (row i = global id i)
    off_attrs  i32 num_parts[n], i16 year[n], i32 theme_id[n]   (bb_upload_attrs columns)
    off_names  UTF-8 JSON list of set_num strings (row order)

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
VERSION = 1
_HDR = struct.Struct("<4sIQIIQQQQ")
_ALIGN = 4096


def _align(x: int) -> int:
    return (x + _ALIGN - 1) // _ALIGN * _ALIGN


def write_index(path: str, set_nums: Sequence[str], rows: np.ndarray, num_parts=None, year=None, theme_id=None,
                unit_norm: bool = False) -> None:
    """Write rows (n×d, stored as f32) and the optional attribute columns."""
    rows = np.asarray(rows)
    n, d = rows.shape
    if len(set_nums) != n:
        raise ValueError("one set_num per row")
    names = json.dumps([str(s) for s in set_nums]).encode()
    off_rows = _align(_HDR.size)
    off_attrs = _align(off_rows + n * d * 4)
    has_attrs = num_parts is not None
    off_names = _align(off_attrs + (n * 10 if has_attrs else 0))
    flags = (1 if unit_norm else 0) | (2 if has_attrs else 0)
    with open(path, "wb") as f:
        f.write(_HDR.pack(MAGIC, VERSION, n, d, flags, off_rows, off_attrs, off_names, len(names)))
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


class IndexFile:
    """A mapped index file: ``rows`` (np.memmap f32 n×d), ``set_nums``, and the attribute
    columns (or None)."""

    def __init__(self, path: str):
        size = os.path.getsize(path)
        with open(path, "rb") as f:
            hdr = f.read(_HDR.size)
        if len(hdr) < _HDR.size:
            raise ValueError(f"{path}: truncated header")
        magic, ver, n, d, flags, off_rows, off_attrs, off_names, names_bytes = _HDR.unpack(hdr)
        if magic != MAGIC or ver != VERSION:
            raise ValueError(f"{path}: not a brickrec index file (v{VERSION})")
        has_attrs = bool(flags & 2)
        if (off_rows + n * d * 4 > size or (has_attrs and off_attrs + n * 10 > size)
                or off_names + names_bytes > size):
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

    def load_into(self, index, present: Optional[np.ndarray] = None):
        """Upload the rows (and attributes) into an ``ItemIndex`` straight from the mapping."""
        index.upload_items(self.rows, prenormalized=self.unit_norm, present=present)
        if self.num_parts is not None:
            index.upload_attrs(self.num_parts, self.year, self.theme_id)
        return index


def open_index(path: str) -> IndexFile:
    return IndexFile(path)
