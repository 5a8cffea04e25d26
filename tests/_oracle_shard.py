"""CPU stand-in for one shard of ``brickrec.ItemIndex`` in the key-list form used by the
sharded search (``search_keys`` / ``finalize`` / ``get_rows``) — TEST INFRASTRUCTURE ONLY.

Keys follow the C-ABI exactly: ``(ord(fp32 score) << 32) | (0xFFFFFFFF - gid)``, stored as
int64 bit patterns. This lets the gloo tests check the orchestration of
``brickrec.distributed.ShardedIndex`` on CPU: row blocks, id offsets, mask and exclusion
slicing, query-row assembly and gather layout. The device kernels behind the same calls
are checked on the GPU (tests/test_gpu_parity.py::test_sharded_merge).
"""
import numpy as np
import torch

from oracle import restatement as R


def ord_of(f32):
    u = np.asarray(f32, np.float32).view(np.uint32).astype(np.uint64)
    neg = (u & 0x80000000) != 0
    return np.where(neg, (~u) & 0xFFFFFFFF, u | 0x80000000).astype(np.uint64)


def float_of_ord(o):
    o = np.asarray(o, np.uint64)
    pos = (o & 0x80000000) != 0
    u = np.where(pos, o & 0x7FFFFFFF, (~o) & 0xFFFFFFFF).astype(np.uint32)
    return u.view(np.float32)


def make_keys(scores, gids):
    k = (ord_of(scores) << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - np.asarray(gids, np.uint64))
    return k.view(np.int64)


def split_keys(keys):
    u = np.asarray(keys, np.int64).view(np.uint64)
    gid = (np.uint64(0xFFFFFFFF) - (u & np.uint64(0xFFFFFFFF))).astype(np.int64)
    return float_of_ord(u >> np.uint64(32)), gid


class OracleShard:
    def __init__(self, id_offset=0):
        self.off = int(id_offset)
        self.x = self.f = None
        self.present = self.cf_present = None
        self.d = 0

    def upload_items(self, rows, prenormalized=False, present=None):
        x = np.asarray(rows, np.float32)
        self.x = x if prenormalized else R.normalize_rows(x.astype(np.float64)).astype(np.float32)
        self.d = x.shape[1]
        self.present = np.ones(len(x), bool) if present is None else np.asarray(present, bool)

    def upload_cf(self, f, present=None):
        self.f = np.asarray(f, np.float32)
        self.cf_present = np.ones(len(self.f), bool) if present is None else np.asarray(present, bool)

    def get_rows(self, ids):
        ids = np.asarray(ids.cpu() if hasattr(ids, "cpu") else ids, np.int64) - self.off
        out = np.zeros((len(ids), self.d), np.float32)
        ok = (ids >= 0) & (ids < len(self.x))
        out[ok] = self.x[ids[ok]]
        return torch.from_numpy(out)

    @staticmethod
    def _bits(t, n):
        if t is None:
            return None
        w = np.ascontiguousarray(t.cpu().numpy()).view(np.uint32)
        return np.unpackbits(w.view(np.uint8), axis=-1, bitorder="little")[..., :n].astype(bool)

    def key_lens(self, mode, k, k_side=0):
        ks = k_side or 2 * k
        return {"semantic": (1, k), "cf": (1, k), "similar": (1, k + 1), "hybrid": (2, ks + 1)}[mode]

    def _side(self, scores, ok, kint):
        i, s = R.topk_indices(scores.astype(np.float32), kint, ok)
        out = np.zeros(kint, np.int64)
        out[: len(i)] = make_keys(s, i + self.off)
        return out

    def search_keys(self, mode, k, *, q_rows=None, q_items=None, q_cf=None, mask=None, excl=None, k_side=0):
        sides, kint = self.key_lens(mode, k, k_side)
        n = len(self.x)
        m = self._bits(mask, n)
        e = self._bits(excl, n)
        B = int((q_rows if q_rows is not None else q_cf).shape[0])
        keys = np.zeros((sides, B, kint), np.int64)
        maxk = np.zeros(B, np.int64)
        for b in range(B):
            if mode in ("semantic", "similar", "hybrid"):
                q = q_rows[b].cpu().numpy().astype(np.float32)
                if mode == "semantic":
                    q = R.normalize_rows(q[None].astype(np.float64))[0].astype(np.float32)
                sim = (self.x @ q).astype(np.float32)
                ok = self.present.copy() if m is None else self.present & m
                keys[0, b] = self._side(sim, ok, kint)
                if mode != "semantic" and self.present.any():
                    p = np.where(self.present, sim, -np.inf)
                    j = int(np.argmax(p))
                    maxk[b] = make_keys([sim[j]], [j + self.off])[0]
            if mode in ("cf", "hybrid"):
                sc = (self.f @ q_cf[b].cpu().numpy().astype(np.float32)).astype(np.float32)
                ok = self.cf_present.copy()
                if m is not None:
                    ok &= m
                if e is not None:
                    ok &= ~e[b]
                keys[sides - 1, b] = self._side(sc, ok, kint)
        return torch.from_numpy(keys), torch.from_numpy(maxk)

    def finalize(self, mode, k, keys, max_keys, n_parts, *, k_side=0, w_content=0.4, w_cf=0.6):
        """Python statement of finalize_kernel (csrc/misc.hip)."""
        keys = keys.cpu().numpy()          # [P, sides, B, kint]
        mk = max_keys.cpu().numpy()        # [P, B]
        P, sides, B, kint = keys.shape
        drop = mode in ("similar", "hybrid")
        ks = k_side or 2 * k
        sc = np.zeros((B, k), np.float32)
        ids = np.full((B, k), -1, np.int64)
        cnt = np.zeros(B, np.int32)
        for b in range(B):
            lists = []
            for s in range(sides):
                u = keys[:, s, b, :].reshape(-1).view(np.uint64)
                u = np.sort(u[u != 0])[::-1]
                if s == 0 and drop:
                    g = mk[:, b].view(np.uint64).max()
                    if len(u) and g and u[0] == g:
                        u = u[1:]
                lists.append(u[: (ks if mode == "hybrid" else k)])
            if mode != "hybrid":
                s_, i_ = split_keys(lists[0].view(np.int64))
            else:
                cs, ci = split_keys(lists[0].view(np.int64))
                fs, fi = split_keys(lists[1].view(np.int64))
                if len(ci) and len(fi):
                    i_, s_ = R.union_blend(ci, cs.astype(np.float64), fi, fs.astype(np.float64), w_content, w_cf, k)
                elif len(ci):
                    i_, s_ = ci[:k], cs[:k]
                else:
                    i_, s_ = fi[:k], fs[:k]
            c = min(k, len(i_))
            ids[b, :c] = i_[:c]
            sc[b, :c] = s_[:c]
            cnt[b] = c
        return torch.from_numpy(sc), torch.from_numpy(ids), torch.from_numpy(cnt)
