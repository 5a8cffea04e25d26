"""Item-index file (brickrec/indexfile.py): round trip of rows, attributes and names through
the mapped file, corrupt-file rejection, and (GPU) a search over an index uploaded straight
from the mapping equals one uploaded from memory."""
import numpy as np
import pytest

from oracle import restatement as R


def test_roundtrip(tmp_path):
    from brickrec.indexfile import open_index, write_index
    rng = np.random.default_rng(3)
    x = R.unit_rows(1000, 96, 5)
    parts = rng.integers(1, 6000, 1000)
    year = rng.integers(1949, 2025, 1000)
    theme = rng.integers(0, 400, 1000)
    names = [f"{i}-1" for i in range(1000)]
    p = str(tmp_path / "items.bbix")
    write_index(p, names, x, parts, year, theme, unit_norm=True)
    f = open_index(p)
    assert f.n == 1000 and f.d == 96 and f.unit_norm and f.set_nums == names
    np.testing.assert_array_equal(np.asarray(f.rows), x.astype(np.float32))
    np.testing.assert_array_equal(f.num_parts, parts)
    np.testing.assert_array_equal(f.year, year)
    np.testing.assert_array_equal(f.theme_id, theme)
    q = open_index(str(_write_plain(tmp_path)))
    assert q.num_parts is None and not q.unit_norm


def _write_plain(tmp_path):
    from brickrec.indexfile import write_index
    p = tmp_path / "plain.bbix"
    write_index(str(p), ["a", "b"], np.eye(2, 8))
    return p


def test_rejects_bad_files(tmp_path):
    from brickrec.indexfile import open_index
    p = _write_plain(tmp_path)
    b = bytearray(p.read_bytes())
    (tmp_path / "magic").write_bytes(b"XXXX" + bytes(b[4:]))
    with pytest.raises(ValueError):
        open_index(str(tmp_path / "magic"))
    (tmp_path / "short").write_bytes(bytes(b[:5000]))
    with pytest.raises(ValueError):
        open_index(str(tmp_path / "short"))


@pytest.mark.gpu
def test_mapped_upload_search(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import brickrec
    from brickrec.indexfile import open_index, write_index
    x = R.unit_rows(20000, 384, 7)
    q = R.unit_rows(64, 384, 8)
    p = str(tmp_path / "items.bbix")
    write_index(p, [str(i) for i in range(len(x))], x, unit_norm=True)
    a = open_index(p).load_into(brickrec.ItemIndex(dtype="f32"))
    b = brickrec.ItemIndex(dtype="f32")
    b.upload_items(x.astype(np.float32), prenormalized=True)
    ra, rb = a.search("semantic", 20, q_rows=q), b.search("semantic", 20, q_rows=q)
    for u, v in zip(ra, rb):
        assert np.array_equal(u, v)
    ri, rs = R.topk_indices(R.cosine_scores(q[:1], x)[0].astype(np.float64), 20)
    assert list(ra[1][0]) == list(ri)
