"""Small-batch debugging on the GPU box: the hybrid request of test_hybrid_requests run side by
side on both paths, each side alone (similar / cf) against an f64 recompute, and the hybrid
key lists (BB_Q_OUT_KEYS) compared entry by entry.   python tools/sq_debug.py [B ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brickbrain-rec-engine_amd"))
sys.path.insert(0, ROOT)
from oracle import restatement as R  # noqa: E402


def exact(rows, q, k, allowed, drop=False):
    s = (rows.astype(np.float64) @ q.astype(np.float64)).astype(np.float32)
    ok = allowed.copy()
    if drop:
        ok[int(np.argmax(s))] = False
    i = np.flatnonzero(ok)
    o = np.lexsort((i, -s[i]))[:k]
    return i[o]


def run(idx, v, *a, **kw):
    idx.set_option("small_batch", v)
    try:
        return idx.search(*a, **kw)
    finally:
        idx.set_option("small_batch", -1)


def main():
    import torch
    import brickrec
    n, d, r = 25216, 384, 50
    for B in [int(b) for b in sys.argv[1:]] or [1, 3]:
        rng = np.random.default_rng(100 + B)
        x = R.unit_rows(n, d, 1234)
        f = rng.normal(0, 0.1, (n, r)).astype(np.float32)
        idx = brickrec.ItemIndex(dtype="f32")
        idx.upload_items(x, prenormalized=True)
        pres = rng.random(n) < 0.8
        idx.upload_cf(f, present=pres)
        liked = rng.choice(n, B, replace=False)
        u = rng.normal(0, 0.1, (B, r)).astype(np.float32)
        mask = rng.random(n) < 0.2
        rated = rng.random((B, n)) < 0.002
        rows = idx.get_rows(np.arange(n))
        for k in (10, 50):
            for mode, kw in (("similar", dict(q_items=liked, mask=mask)),
                             ("cf", dict(q_cf=u, mask=mask, excl=rated)),
                             ("hybrid", dict(q_items=liked, q_cf=u, mask=mask, excl=rated))):
                res = [run(idx, v, mode, k, **kw) for v in (0, 1)]
                same = all(np.array_equal(res[0][j], res[1][j]) for j in (1, 2))
                msg = f"B={B} k={k} {mode:8s} paths equal={same}"
                if mode != "hybrid":
                    for v in (0, 1):
                        ok = 0
                        for b in range(B):
                            if mode == "similar":
                                ri = exact(rows, rows[liked[b]], k, mask, drop=True)
                            else:
                                ri = exact(f, u[b], k, mask & pres & ~rated[b])
                            ok += list(res[v][1][b][:len(ri)]) == list(ri)
                        msg += f" v{v} exact {ok}/{B}"
                print(msg, flush=True)
        for k in (5, 10, 11, 16, 20, 21, 24, 30, 40):
            res = [run(idx, v, "cf", k, q_cf=u) for v in (0, 1)]
            ok = [sum(list(res[v][1][b]) == list(exact(f, u[b], k, pres)) for b in range(B)) for v in (0, 1)]
            print(f"B={B} cf unmasked k={k}: exact v0 {ok[0]}/{B} v1 {ok[1]}/{B}", flush=True)
        outs = {}
        for v in (0, 1):
            idx.set_option("small_batch", v)
            outs[v] = idx.search_keys("hybrid", 10, q_items=torch.from_numpy(liked).cuda(),
                                      q_cf=torch.from_numpy(u).cuda())
            idx.set_option("small_batch", -1)
        torch.cuda.synchronize()
        k0, k1 = outs[0][0].cpu().numpy().view(np.uint64), outs[1][0].cpu().numpy().view(np.uint64)
        print(f"B={B} keys shape {k0.shape} equal {np.array_equal(k0, k1)} max equal "
              f"{torch.equal(outs[0][1], outs[1][1])}", flush=True)
        if not np.array_equal(k0, k1):
            for s in range(k0.shape[0]):
                for b in range(min(B, 2)):
                    a0, a1 = k0[s, b], k1[s, b]
                    bad = np.flatnonzero(a0 != a1)
                    if s == 1 and b == 0:
                        g = lambda a: [int(0xFFFFFFFF - (int(t) & 0xFFFFFFFF)) for t in a[:6]]
                        print("  exact cf top", list(exact(f, u[0], 6, pres)), "v0", g(a0), "v1", g(a1), flush=True)
                        sim = exact(rows, rows[liked[0]], 200, np.ones(n, bool))
                        pos = {int(t): j for j, t in enumerate(sim)}
                        print("  v1 cf items' ranks in the content top-200:", [pos.get(t, -1) for t in g(a1)],
                              flush=True)
                        cfr = exact(f, u[0], n, pres)
                        posc = {int(t): j for j, t in enumerate(cfr)}
                        print("  v1 cf items' exact cf ranks:", [posc.get(t, -1) for t in g(a1)], flush=True)
                    if len(bad):
                        print(f"  side {s} row {b}: {len(bad)} differ, first at {bad[0]}: "
                              f"{a0[bad[0]] >> 32:#x}/{a0[bad[0]] & 0xffffffff} vs "
                              f"{a1[bad[0]] >> 32:#x}/{a1[bad[0]] & 0xffffffff}", flush=True)
        idx.close()


if __name__ == "__main__":
    main()
