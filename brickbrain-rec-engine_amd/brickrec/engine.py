"""Device-resident item index: the Python face of libbrickrec.

``ItemIndex`` owns one ``bb_index`` handle (one HIP stream, device copies of the item
matrix, CF factors and attribute columns) and exposes the batched search.  Inputs may be
numpy arrays (host; results come back as numpy) or torch CUDA tensors (device; results
are torch tensors on the same device, nothing synchronises).  Calls are serialised per
handle with a lock, matching the reference's single shared engine
(recommendation_api.py:44-67).
"""
from __future__ import annotations

import ctypes as C
import threading
import weakref
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib as L

MODES = {"semantic": L.BB_MODE_SEMANTIC, "similar": L.BB_MODE_SIMILAR, "cf": L.BB_MODE_CF,
         "hybrid": L.BB_MODE_HYBRID}
INT32_MIN, INT32_MAX = -(2 ** 31), 2 ** 31 - 1


def bits_from_bool(mask) -> np.ndarray:
    """bool [..., n] -> uint32 words [..., ceil(n/32)], bit i of word w = item 32w+i."""
    m = np.asarray(mask, dtype=bool)
    n = m.shape[-1]
    nw = (n + 31) // 32
    pad = np.zeros(m.shape[:-1] + (nw * 32,), dtype=bool)
    pad[..., :n] = m
    return np.ascontiguousarray(np.packbits(pad, axis=-1, bitorder="little").view(np.uint32))


def bool_from_bits(words, n: int) -> np.ndarray:
    w = np.ascontiguousarray(np.asarray(words, dtype=np.uint32))
    return np.unpackbits(w.view(np.uint8), axis=-1, bitorder="little")[..., :n].astype(bool)


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _np_dtype_code(a: np.ndarray) -> int:
    if a.dtype == np.float32:
        return L.BB_F32
    if a.dtype == np.float64:
        return L.BB_F64
    raise TypeError(f"unsupported row dtype {a.dtype}")


def _null(stream) -> int:
    """torch's default stream has handle 0: tell the library to use the null stream instead
    of its own (NULL in bb_query.stream means 'the handle's stream')."""
    return L.BB_Q_NULL_STREAM if int(stream.cuda_stream) == 0 else 0


def _torch_dtype_code(t) -> int:
    import torch
    return {torch.float32: L.BB_F32, torch.float64: L.BB_F64, torch.bfloat16: L.BB_BF16}[t.dtype]


@dataclass
class Predicate:
    """On-device form of the hard-constraint WHERE clause (see include/brickrec.h)."""
    parts_min: int = INT32_MIN
    parts_max: int = INT32_MAX
    year_min: int = INT32_MIN
    year_max: int = INT32_MAX
    theme_mode: int = 0                 # 0 none, 1 require, 2 exclude
    theme_ids: Sequence[int] = ()
    excluded_items: Sequence[int] = ()  # global ids


class _Plan:
    """A prepared search (bb_plan_create): calling it replays the recorded launches
    (bb_plan_launch).  It holds its inputs, outputs and index alive; close() (or garbage
    collection, or closing the index) destroys the plan and its private view."""

    is_plan = True  # run() replays a bb_plan (the bb_search closure says False)

    def __init__(self, lib, handle, root, keep):
        self._lib, self._p, self._root, self._keep = lib, handle, root, keep
        self._launch = lib.bb_plan_launch
        if not hasattr(root, "_plans"):
            root._plans = weakref.WeakSet()
        root._plans.add(self)

    def __call__(self):
        rc = self._launch(self._p)
        if rc:
            L.check(rc, "bb_plan_launch")

    def close(self):
        p, self._p = getattr(self, "_p", None), None
        if not p:
            return
        root = self._root
        rc = self._lib.bb_plan_destroy(p)
        with root._mu:
            root._views -= 1
        getattr(root, "_plans", set()).discard(self)
        L.check(rc, "bb_plan_destroy")

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ItemIndex:
    def __init__(self, device: int = 0, dtype: str = "f32", id_offset: int = 0,
                 workspace_bytes: int = 0):
        self._lib = L.load()
        self.dtype = dtype
        self.device = device
        self.id_offset = int(id_offset)
        code = {"f32": L.BB_F32, "bf16": L.BB_BF16}[dtype]
        desc = L.bb_desc(device, code, self.id_offset, int(workspace_bytes))
        h = C.c_void_p()
        L.check(self._lib.bb_create(C.byref(desc), C.byref(h)), "bb_create")
        self._h = h
        # re-entrant: close() can run from __del__ (cyclic GC) on a thread already holding this
        # lock inside view() / search(), and takes the view's and then the base's lock
        self._mu = threading.RLock()
        self.n_items = 0
        self.d = 0
        self.r = 0

    # ------------------------------------------------------------------ lifetime
    def view(self) -> "ItemIndex":
        """A second handle over this index's resident rows (bb_create_view): its own HIP stream
        and workspace, no second copy of the items — for keeping several batches in flight.
        Close the views before closing or re-uploading this index."""
        v = ItemIndex.__new__(ItemIndex)
        v._lib, v.dtype, v.device, v.id_offset = self._lib, self.dtype, self.device, self.id_offset
        h = C.c_void_p()
        with self._mu:  # the view count changes under the base's lock (view(), close())
            L.check(self._lib.bb_create_view(self._h, C.byref(h)), "bb_create_view")
            self._views = getattr(self, "_views", 0) + 1
        v._h = h
        v._mu = threading.RLock()
        v.n_items, v.d, v.r = self.n_items, self.d, self.r
        v._base = self  # keeps the base alive while the view is
        return v

    def close(self):
        mu = getattr(self, "_mu", None)
        if mu is None:
            return
        for p in list(getattr(self, "_plans", ())):
            p.close()
        with mu:
            if not getattr(self, "_h", None):
                return
            if getattr(self, "_views", 0):
                raise L.BrickrecError("close this index's views first")
            L.check(self._lib.bb_destroy(self._h), "bb_destroy")
            self._h = None
        base = getattr(self, "_base", None)
        if base is not None:
            with base._mu:
                base._views -= 1

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ uploads
    def upload_items(self, rows, prenormalized: bool = False, present: Optional[np.ndarray] = None):
        """Upload the item matrix (n×d).  numpy f32/f64 (host) or torch CUDA f32/bf16/f64.
        present: bool [n] rows that exist in the content item space (None = all)."""
        bits = bits_from_bool(present) if present is not None else None
        bp = bits.ctypes.data if bits is not None else None
        with self._mu:
            if _is_torch(rows):
                import torch
                rows = rows.contiguous()
                # the library converts on its own stream: the rows must be complete first
                torch.cuda.current_stream(rows.device).synchronize()
                n, d = rows.shape
                rc = self._lib.bb_upload_items(self._h, rows.data_ptr(), n, d, _torch_dtype_code(rows),
                                               int(prenormalized), L.BB_DEVICE, bp)
            else:
                rows = np.ascontiguousarray(rows)
                if rows.dtype not in (np.float32, np.float64):
                    rows = rows.astype(np.float64)
                n, d = rows.shape
                rc = self._lib.bb_upload_items(self._h, rows.ctypes.data, n, d, _np_dtype_code(rows),
                                               int(prenormalized), L.BB_HOST, bp)
            L.check(rc, "bb_upload_items")
            self.n_items, self.d = int(n), int(d)

    def upload_cf(self, item_factors: np.ndarray, present: Optional[np.ndarray] = None):
        """CF item factors (n×r, same row space as the items) + presence mask (bool n)."""
        f = np.ascontiguousarray(item_factors)
        if f.dtype not in (np.float32, np.float64):
            f = f.astype(np.float64)
        bits = bits_from_bool(present) if present is not None else None
        with self._mu:
            L.check(self._lib.bb_upload_cf(self._h, f.ctypes.data, f.shape[1], _np_dtype_code(f),
                                           bits.ctypes.data if bits is not None else None),
                    "bb_upload_cf")
            self.r = int(f.shape[1])

    def upload_attrs(self, num_parts, year, theme_id):
        p = np.ascontiguousarray(num_parts, dtype=np.int32)
        y = np.ascontiguousarray(np.clip(year, -32768, 32767), dtype=np.int16)
        t = np.ascontiguousarray(theme_id, dtype=np.int32)
        with self._mu:
            L.check(self._lib.bb_upload_attrs(self._h, p.ctypes.data, y.ctypes.data, t.ctypes.data),
                    "bb_upload_attrs")

    def eval_mask_bits(self, pred: Predicate):
        """Evaluate a predicate on the device -> the mask as a device bitset (torch int32
        [ceil(n/32)] on this index's device), ready to pass to search / search_keys."""
        import torch
        ids = np.asarray(list(pred.theme_ids), dtype=np.int64)
        nbits = int(ids.max()) + 1 if ids.size else 0
        tb = bits_from_bool(np.isin(np.arange(nbits), ids)) if nbits else np.zeros(1, np.uint32)
        ex = np.ascontiguousarray(np.asarray(list(pred.excluded_items), dtype=np.int64))
        bp = L.bb_predicate(int(pred.parts_min), int(pred.parts_max), int(pred.year_min),
                            int(pred.year_max), int(pred.theme_mode), nbits, tb.ctypes.data,
                            ex.ctypes.data if ex.size else None, int(ex.size))
        out = torch.zeros(((self.n_items + 31) // 32,), dtype=torch.int32, device=torch.device("cuda", self.device))
        torch.cuda.current_stream(out.device).synchronize()
        with self._mu:
            L.check(self._lib.bb_eval_mask(self._h, C.byref(bp), out.data_ptr(), L.BB_DEVICE), "bb_eval_mask")
        return out

    def eval_mask(self, pred: Predicate) -> np.ndarray:
        """Evaluate a predicate on the device -> bool mask over the local items."""
        ids = np.asarray(list(pred.theme_ids), dtype=np.int64)
        nbits = int(ids.max()) + 1 if ids.size else 0
        tb = bits_from_bool(np.isin(np.arange(nbits), ids)) if nbits else np.zeros(1, np.uint32)
        ex = np.ascontiguousarray(np.asarray(list(pred.excluded_items), dtype=np.int64))
        bp = L.bb_predicate(int(pred.parts_min), int(pred.parts_max), int(pred.year_min),
                            int(pred.year_max), int(pred.theme_mode), nbits, tb.ctypes.data,
                            ex.ctypes.data if ex.size else None, int(ex.size))
        out = np.zeros((self.n_items + 31) // 32, dtype=np.uint32)
        with self._mu:
            L.check(self._lib.bb_eval_mask(self._h, C.byref(bp), out.ctypes.data, L.BB_HOST),
                    "bb_eval_mask")
        return bool_from_bits(out, self.n_items)

    # ------------------------------------------------------------------ search
    def _query(self, mode, k, B, k_side, where, q_rows, q_dtype, q_items, q_cf, q_cf_dtype, mask,
               excl, w_content, w_cf, stream, flags, mask_count=0):
        return L.bb_query(MODES[mode] if isinstance(mode, str) else mode, flags, B, k, k_side, where,
                          q_rows, q_dtype, q_items, q_cf, q_cf_dtype, mask, excl,
                          float(w_content), float(w_cf), stream, int(mask_count or 0))

    def search(self, mode: str, k: int, *, q_rows=None, q_items=None, q_cf=None, mask=None,
               excl=None, k_side: int = 0, w_content: float = 0.4, w_cf: float = 0.6,
               stream=None, out=None, mask_count: int = 0):
        """Batched top-k.  Returns (scores [B,k] f32, ids [B,k] i64, counts [B] i32).

        mask: bool [n] (or uint32 words) — items allowed (valid_set_filter); excl: bool
        [B, n] (or words) — per-query excluded items (CF: rated).  Torch CUDA inputs run
        fully asynchronously on `stream` (default: torch's current stream).  mask_count: the
        number of allowed items of a device (torch int32 words) mask, when known — the
        length of the reference's valid_set_nums; host and bool masks are counted here or
        by the library (bb_query.mask_count, constraint-first search)."""
        first = next(x for x in (q_rows, q_items, q_cf) if x is not None)
        if _is_torch(first):
            return self._search_torch(mode, k, q_rows, q_items, q_cf, mask, excl, k_side, w_content,
                                      w_cf, stream, out, mask_count)
        B = int(np.asarray(first).shape[0])
        keep = []

        def arr(x, dt=None):
            if x is None:
                return None, 0
            a = np.ascontiguousarray(x if dt is None else np.asarray(x, dtype=dt))
            keep.append(a)
            return a.ctypes.data, (_np_dtype_code(a) if a.dtype in (np.float32, np.float64) else 0)

        qr, qd = arr(q_rows if q_rows is None or np.asarray(q_rows).dtype in (np.float32, np.float64)
                     else np.asarray(q_rows, np.float64))
        qi, _ = arr(q_items, np.int64)
        qc, qcd = arr(q_cf if q_cf is None or np.asarray(q_cf).dtype in (np.float32, np.float64)
                      else np.asarray(q_cf, np.float64))
        mw = None if mask is None else (np.asarray(mask, np.uint32) if np.asarray(mask).dtype == np.uint32
                                        else bits_from_bool(mask))
        ew = None if excl is None else (np.asarray(excl, np.uint32) if np.asarray(excl).dtype == np.uint32
                                        else bits_from_bool(excl))
        mp, _ = arr(mw)
        ep, _ = arr(ew)
        scores = np.zeros((B, k), np.float32)
        ids = np.zeros((B, k), np.int64)
        counts = np.zeros(B, np.int32)
        q = self._query(mode, k, B, k_side, L.BB_HOST, qr, qd, qi, qc, qcd, mp, ep, w_content, w_cf,
                        None, 0)
        res = L.bb_result(scores.ctypes.data, ids.ctypes.data, counts.ctypes.data, L.BB_HOST, None, None)
        with self._mu:
            L.check(self._lib.bb_search(self._h, C.byref(q), C.byref(res)), "bb_search")
        return scores, ids, counts

    def _search_torch(self, mode, k, q_rows, q_items, q_cf, mask, excl, k_side, w_content, w_cf,
                      stream, out, mask_count=0):
        import torch
        first = next(x for x in (q_rows, q_items, q_cf) if x is not None)
        dev = first.device
        B = int(first.shape[0])
        keep = []

        def ptr(t, dt=None):
            if t is None:
                return None
            t = t.to(dev) if dt is None else t.to(dev, dt)
            t = t.contiguous()
            keep.append(t)
            return t.data_ptr()

        if mask is not None and mask.dtype == torch.bool:
            mb = mask.cpu().numpy()
            mask_count = int(np.count_nonzero(mb[: self.n_items]))
            mask = torch.from_numpy(bits_from_bool(mb).view(np.int32)).to(dev)
        if excl is not None and excl.dtype == torch.bool:
            excl = torch.from_numpy(bits_from_bool(excl.cpu().numpy()).view(np.int32)).to(dev)
        if out is None:
            out = (torch.empty((B, k), dtype=torch.float32, device=dev),
                   torch.empty((B, k), dtype=torch.int64, device=dev),
                   torch.empty((B,), dtype=torch.int32, device=dev))
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        q = self._query(mode, k, B, k_side, L.BB_DEVICE,
                        ptr(q_rows), _torch_dtype_code(q_rows) if q_rows is not None else 0,
                        ptr(q_items, torch.int64),
                        ptr(q_cf), _torch_dtype_code(q_cf) if q_cf is not None else 0,
                        ptr(mask), ptr(excl), w_content, w_cf, s.cuda_stream, _null(s), mask_count)
        res = L.bb_result(out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), L.BB_DEVICE,
                          None, None)
        with self._mu:
            L.check(self._lib.bb_search(self._h, C.byref(q), C.byref(res)), "bb_search")
        return out

    def prepared_search(self, mode: str, k: int, *, q_rows=None, q_items=None, q_cf=None,
                        mask=None, excl=None, k_side: int = 0, w_content=0.4, w_cf=0.6,
                        stream=None, plan: bool = True, mask_count: int = 0):
        """A repeated device-resident search (the serving loop; bench).  All inputs must be
        torch CUDA tensors of the right dtypes; returns (run, outputs): each run() searches
        the inputs' current contents into the same outputs.  With plan=True (default) run is a
        bb_plan (include/brickrec.h): the host logic ran once, run() replays the launches; with
        plan=False, or a search that synchronises with the host mid-way (bb_plan_create's
        BB_E_HOSTSYNC: the streaming top-K), run() calls bb_search.  run.is_plan says which.
        Any other plan refusal raises.  A plan may be called from several threads (the C-ABI
        serialises its launches)."""
        import torch
        first = next(x for x in (q_rows, q_items, q_cf) if x is not None)
        dev, B = first.device, int(first.shape[0])
        out = (torch.empty((B, k), dtype=torch.float32, device=dev),
               torch.empty((B, k), dtype=torch.int64, device=dev),
               torch.empty((B,), dtype=torch.int32, device=dev))
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        keep = [t for t in (q_rows, q_items, q_cf, mask, excl) if t is not None]
        keep.append(s)  # a plan's stream must outlive it (bb_plan_destroy synchronises it)
        q = self._query(mode, k, B, k_side, L.BB_DEVICE,
                        q_rows.data_ptr() if q_rows is not None else None,
                        _torch_dtype_code(q_rows) if q_rows is not None else 0,
                        q_items.data_ptr() if q_items is not None else None,
                        q_cf.data_ptr() if q_cf is not None else None,
                        _torch_dtype_code(q_cf) if q_cf is not None else 0,
                        mask.data_ptr() if mask is not None else None,
                        excl.data_ptr() if excl is not None else None, w_content, w_cf,
                        s.cuda_stream, _null(s), mask_count)
        res = L.bb_result(out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), L.BB_DEVICE, None, None)
        if plan:
            # bb_plan_create: the host side of the search runs once; each call replays its
            # launches.  Searches that synchronise with the host (the streaming top-K) refuse a
            # plan (BB_E_HOSTSYNC) and keep the bb_search call below; nothing else falls back.
            root = getattr(self, "_base", None) or self
            ph = C.c_void_p()
            with root._mu, self._mu:
                rc = self._lib.bb_plan_create(self._h, C.byref(q), C.byref(res), C.byref(ph))
                if rc == 0:
                    root._views = getattr(root, "_views", 0) + 1   # the plan's private view
            if rc == 0:
                p = _Plan(self._lib, ph, root, (keep, q, res, self))
                return p, out
            if rc != L.BB_E_HOSTSYNC:
                L.check(rc, "bb_plan_create")
        fn, h, qp, rp = self._lib.bb_search, self._h, C.byref(q), C.byref(res)

        def run():
            rc = fn(h, qp, rp)
            if rc:
                L.check(rc, "bb_search")
        run._keep = (keep, q, res, self)  # buffers, structs and the index handle live as long as the closure
        run.is_plan = False
        return run, out

    # ------------------------------------------------------------------ sharded search
    def key_lens(self, mode: str, k: int, k_side: int = 0) -> Tuple[int, int]:
        q = self._query(mode, k, 1, k_side, L.BB_DEVICE, None, 0, None, None, 0, None, None, 0, 0, None, 0)
        s, ki = C.c_int32(), C.c_int32()
        L.check(self._lib.bb_key_lens(C.byref(q), C.byref(s), C.byref(ki)), "bb_key_lens")
        return s.value, ki.value

    def search_keys(self, mode: str, k: int, *, q_rows=None, q_items=None, q_cf=None, mask=None,
                    excl=None, k_side: int = 0, stream=None):
        """Local candidate lists for a cross-shard merge (torch CUDA in/out):
        keys [sides, B, k_int] u64-as-int64, max_keys [B]."""
        import torch
        first = next(x for x in (q_rows, q_items, q_cf) if x is not None)
        dev, B = first.device, int(first.shape[0])
        sides, kint = self.key_lens(mode, k, k_side)
        keys = torch.zeros((sides, B, kint), dtype=torch.int64, device=dev)
        maxk = torch.zeros((B,), dtype=torch.int64, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        keep = [t for t in (q_rows, q_items, q_cf, mask, excl) if t is not None]
        keep.append(s)  # a plan's stream must outlive it (bb_plan_destroy synchronises it)
        q = self._query(mode, k, B, k_side, L.BB_DEVICE,
                        q_rows.data_ptr() if q_rows is not None else None,
                        _torch_dtype_code(q_rows) if q_rows is not None else 0,
                        q_items.data_ptr() if q_items is not None else None,
                        q_cf.data_ptr() if q_cf is not None else None,
                        _torch_dtype_code(q_cf) if q_cf is not None else 0,
                        mask.data_ptr() if mask is not None else None,
                        excl.data_ptr() if excl is not None else None, 0.4, 0.6, s.cuda_stream,
                        L.BB_Q_OUT_KEYS | _null(s))
        res = L.bb_result(None, None, None, L.BB_DEVICE, keys.data_ptr(), maxk.data_ptr())
        with self._mu:
            L.check(self._lib.bb_search(self._h, C.byref(q), C.byref(res)), "bb_search(keys)")
        del keep
        return keys, maxk

    def finalize(self, mode: str, k: int, keys, max_keys, n_parts: int, *, k_side: int = 0,
                 w_content: float = 0.4, w_cf: float = 0.6, stream=None):
        """Merge gathered shard lists keys [P, sides, B, k_int], max_keys [P, B] -> results."""
        import torch
        B = int(keys.shape[2])
        dev = keys.device
        out = (torch.empty((B, k), dtype=torch.float32, device=dev),
               torch.empty((B, k), dtype=torch.int64, device=dev),
               torch.empty((B,), dtype=torch.int32, device=dev))
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        q = self._query(mode, k, B, k_side, L.BB_DEVICE, None, 0, None, None, 0, None, None,
                        w_content, w_cf, s.cuda_stream, _null(s))
        res = L.bb_result(out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), L.BB_DEVICE, None, None)
        keys = keys.contiguous()
        max_keys = max_keys.contiguous()
        with self._mu:
            L.check(self._lib.bb_finalize(self._h, C.byref(q), keys.data_ptr(), max_keys.data_ptr(),
                                          int(n_parts), C.byref(res)), "bb_finalize")
        return out

    def search_hybrid_sides(self, k: int, *, q_items, q_cf, mask=None, excl=None, k_side: int = 0,
                            w_content: float = 0.4, w_cf: float = 0.6):
        """HYBRID in one device pass with each final item's side membership: bb_search (both
        sides scored and selected in the same search, key lists out) then bb_finalize (rank-0
        drop, union blend wc·c + wcf·cf in f64 on the device).  Host numpy in and out through
        ctypes (no torch): returns (scores [B,k], ids [B,k], counts [B], in_content [B,k] bool,
        in_cf [B,k] bool, side lists [B] of (content ids, CF ids)).  The membership is what
        _combine_recommendations (recommendation_system.py:789-843) builds its reasons from."""
        qi = np.ascontiguousarray(np.asarray(q_items, np.int64))
        B = int(qi.shape[0])
        qc = np.ascontiguousarray(q_cf if np.asarray(q_cf).dtype in (np.float32, np.float64)
                                  else np.asarray(q_cf, np.float64))
        words = lambda m: None if m is None else np.ascontiguousarray(
            np.asarray(m, np.uint32) if np.asarray(m).dtype == np.uint32 else bits_from_bool(m))
        mw, ew = words(mask), words(excl)
        sides_n, kint = self.key_lens("hybrid", k, k_side)
        keys = np.zeros((1, sides_n, B, kint), np.uint64)
        maxk = np.zeros((1, B), np.uint64)
        ptr = lambda a: None if a is None else a.ctypes.data
        q = self._query("hybrid", k, B, k_side, L.BB_HOST, None, 0, qi.ctypes.data, qc.ctypes.data,
                        _np_dtype_code(qc), ptr(mw), ptr(ew), w_content, w_cf, None, L.BB_Q_OUT_KEYS)
        res = L.bb_result(None, None, None, L.BB_HOST, keys.ctypes.data, maxk.ctypes.data)
        sc = np.zeros((B, k), np.float32)
        ids = np.zeros((B, k), np.int64)
        cnt = np.zeros(B, np.int32)
        qf = self._query("hybrid", k, B, k_side, L.BB_HOST, None, 0, None, None, 0, None, None,
                         w_content, w_cf, None, 0)
        resf = L.bb_result(sc.ctypes.data, ids.ctypes.data, cnt.ctypes.data, L.BB_HOST, None, None)
        with self._mu:
            L.check(self._lib.bb_search(self._h, C.byref(q), C.byref(res)), "bb_search(keys)")
            L.check(self._lib.bb_finalize(self._h, C.byref(qf), keys.ctypes.data, maxk.ctypes.data, 1,
                                          C.byref(resf)), "bb_finalize")
        kk, mk = keys[0], maxk[0]
        ks = k_side or 2 * k
        gid = lambda u: (np.uint64(0xFFFFFFFF) - (u & np.uint64(0xFFFFFFFF))).astype(np.int64)
        in_c = np.zeros(ids.shape, bool)
        in_f = np.zeros(ids.shape, bool)
        sides = []
        for b in range(B):
            c = kk[0, b][kk[0, b] != 0]
            if len(c) and mk[b] and c[0] == mk[b]:   # the rank-0 drop finalize applies
                c = c[1:]
            f = kk[1, b][kk[1, b] != 0]
            cs, fs = set(gid(c[:ks]).tolist()), gid(f[:ks])
            in_c[b] = [int(i) in cs for i in ids[b]]
            in_f[b] = np.isin(ids[b], fs)
            sides.append((gid(c[:ks]), fs))
        return sc, ids, cnt, in_c & (ids >= 0), in_f & (ids >= 0), sides

    def get_rows(self, ids):
        """Stored (normalised) rows of global ids: numpy in -> numpy out (f32 view of the
        index dtype: f32, or bf16 widened), torch CUDA int64 in -> torch tensor out."""
        if _is_torch(ids):
            import torch
            dt = torch.float32 if self.dtype == "f32" else torch.bfloat16
            out = torch.empty((int(ids.shape[0]), self.d), dtype=dt, device=ids.device)
            ids = ids.contiguous()
            torch.cuda.current_stream(ids.device).synchronize()  # read on the library's stream
            with self._mu:
                L.check(self._lib.bb_get_rows(self._h, ids.data_ptr(), int(ids.shape[0]), out.data_ptr(),
                                              L.BB_DEVICE), "bb_get_rows")
            return out
        a = np.ascontiguousarray(np.asarray(ids, np.int64))
        if self.dtype == "f32":
            out = np.empty((len(a), self.d), np.float32)
        else:
            out = np.empty((len(a), self.d), np.uint16)
        with self._mu:
            L.check(self._lib.bb_get_rows(self._h, a.ctypes.data, len(a), out.ctypes.data, L.BB_HOST),
                    "bb_get_rows")
        if self.dtype != "f32":
            out = (out.astype(np.uint32) << 16).view(np.float32)
        return out

    # ------------------------------------------------------------------ options
    def set_option(self, option: str, value: int):
        """Tuning knobs: "stream" (-1 auto / 0 off / 1 on), "stream_min_items", "workspace_bytes",
        "stream_refine" (-1 auto / 0 off / 1 on: the two-level streaming bound), "rr_lists" (-1 auto
        / 0 off: bounded candidate lists instead of a score image on one-slab f32 searches),
        "small_batch" (-1 auto / 0 off: the one-pass exact search of batches of <= 16 rows)."""
        code = {"stream": L.BB_OPT_STREAM, "stream_min_items": L.BB_OPT_STREAM_MIN_ITEMS,
                "workspace_bytes": L.BB_OPT_WORKSPACE_BYTES, "stream_refine": L.BB_OPT_STREAM_REFINE,
                "rr_lists": L.BB_OPT_RR_LISTS, "small_batch": L.BB_OPT_SMALL_BATCH,
                "prefilter": L.BB_OPT_PREFILTER}[option]
        with self._mu:
            L.check(self._lib.bb_set_option(self._h, code, int(value)), "bb_set_option")

    # ------------------------------------------------------------------ profiling
    def set_profiling(self, on: bool):
        L.check(self._lib.bb_set_profiling(self._h, int(bool(on))), "bb_set_profiling")

    def profile(self) -> dict:
        p = L.bb_profile()
        with self._mu:
            L.check(self._lib.bb_get_profile(self._h, C.byref(p)), "bb_get_profile")
        return {p.names[i].decode(): {"ms": p.ms[i], "launches": int(p.launches[i])} for i in range(p.n)}
