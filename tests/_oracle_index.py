"""A CPU stand-in for ``brickrec.ItemIndex`` built on the oracle — TEST INFRASTRUCTURE ONLY.

Tests inject it through ``Engine(index_factory=OracleIndex)``, so that they can exercise
the drop-in recommenders, the constraint filter and the FastAPI routes on a machine
without a GPU. The product code never imports it: ``Engine`` defaults to the HIP
``ItemIndex`` and has no fallback. On the GPU box the same tests run against the real
index (tests/test_dropin_gpu.py).
"""
import numpy as np

from oracle import restatement as R


class OracleIndex:
    def __init__(self):
        self.x = None
        self.present = None
        self.f = None
        self.cf_present = None
        self.attrs = None

    def upload_items(self, rows, prenormalized=False, present=None):
        x = np.asarray(rows, np.float64)
        self.x = x if prenormalized else R.normalize_rows(x)
        self.present = np.ones(len(x), bool) if present is None else np.asarray(present, bool)

    def upload_cf(self, factors, present=None):
        self.f = np.asarray(factors, np.float64)
        self.cf_present = np.ones(len(self.f), bool) if present is None else np.asarray(present, bool)

    def upload_attrs(self, num_parts, year, theme_id):
        self.attrs = (np.asarray(num_parts), np.asarray(year), np.asarray(theme_id))

    def eval_mask(self, pred):
        parts, year, theme = (a.astype(np.int64) for a in self.attrs)
        m = (parts > 0) & (parts >= pred.parts_min) & (parts <= pred.parts_max)
        m &= (year >= pred.year_min) & (year <= pred.year_max)
        if pred.theme_mode:
            inset = np.isin(theme, list(pred.theme_ids))
            m &= (theme >= 0) & (inset if pred.theme_mode == 1 else ~inset)
        if len(pred.excluded_items):
            m[np.asarray(pred.excluded_items, np.int64)] = False
        return m

    # ------------------------------------------------------------------ search
    def _content(self, q_row, k, mask):
        sim = self.x[q_row] @ self.x.T
        s = np.where(self.present, sim, -np.inf)
        drop = int(np.argmax(s))
        ok = self.present.copy() if mask is None else self.present & np.asarray(mask, bool)
        ok[drop] = False
        return R.topk_indices(sim, k, ok)

    def _cf(self, u, k, mask, excl):
        ok = self.cf_present.copy()
        if mask is not None:
            ok &= np.asarray(mask, bool)
        if excl is not None:
            ok &= ~np.asarray(excl, bool)
        return R.topk_indices(self.f @ np.asarray(u, np.float64), k, ok)

    def search(self, mode, k, *, q_rows=None, q_items=None, q_cf=None, mask=None, excl=None, k_side=0,
               w_content=0.4, w_cf=0.6, stream=None):
        B = len(q_rows if q_rows is not None else q_items if q_items is not None else q_cf)
        sc = np.zeros((B, k), np.float32)
        ids = np.full((B, k), -1, np.int64)
        cnt = np.zeros(B, np.int32)
        for b in range(B):
            eb = None if excl is None else excl[b]
            if mode == "semantic":
                q = R.normalize_rows(np.asarray(q_rows[b:b + 1], np.float64))[0]
                ok = self.present if mask is None else self.present & np.asarray(mask, bool)
                i, s = R.topk_indices(self.x @ q, k, ok)
            elif mode == "similar":
                i, s = self._content(int(q_items[b]), k, mask)
            elif mode == "cf":
                i, s = self._cf(q_cf[b], k, mask, eb)
            else:
                ks = k_side or 2 * k
                ci, cs = self._content(int(q_items[b]), ks, mask)
                fi, fs = self._cf(q_cf[b], ks, mask, eb)
                if len(ci) and len(fi):
                    i, s = R.union_blend(ci, cs, fi, fs, w_content, w_cf, k)
                elif len(ci):
                    i, s = ci[:k], cs[:k]
                else:
                    i, s = fi[:k], fs[:k]
            n = len(i)
            ids[b, :n] = i
            sc[b, :n] = s
            cnt[b] = n
        return sc, ids, cnt

    def search_hybrid_sides(self, k, *, q_items, q_cf, mask=None, excl=None, k_side=0, w_content=0.4, w_cf=0.6):
        B = len(q_items)
        ks = k_side or 2 * k
        sc = np.zeros((B, k), np.float32)
        ids = np.full((B, k), -1, np.int64)
        cnt = np.zeros(B, np.int32)
        in_c = np.zeros((B, k), bool)
        in_f = np.zeros((B, k), bool)
        sides = []
        for b in range(B):
            ci, cs = self._content(int(q_items[b]), ks, mask)
            fi, fs = self._cf(q_cf[b], ks, mask, None if excl is None else excl[b])
            i, s = R.union_blend(ci, cs, fi, fs, w_content, w_cf, k)
            n = len(i)
            ids[b, :n], sc[b, :n], cnt[b] = i, s, n
            in_c[b, :n] = np.isin(i, ci)
            in_f[b, :n] = np.isin(i, fi)
            sides.append((np.asarray(ci, np.int64), np.asarray(fi, np.int64)))
        return sc, ids, cnt, in_c, in_f, sides
