"""G1 (the catalog's 1,934 x 10 content features) on the device index, on the GPU box: the
similar-sets search of test_batch_route through each path, against the golden lists.
    python tools/g1_debug.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brickbrain-rec-engine_amd"))
sys.path.insert(0, ROOT)


def main():
    import brickrec
    g = np.load(os.path.join(ROOT, "tests", "golden", "g1_content.npz"))
    x = g["feat_matrix"]
    idx = brickrec.ItemIndex(dtype="f32")
    idx.upload_items(x)
    q = g["query_rows"][:4]
    for sb in (0, 1):
        idx.set_option("small_batch", sb)
        for k in (5, 50):
            sc, ids, cnt = idx.search("similar", k, q_items=q)
            ok = [list(ids[b]) == list(g["ids_nofilter"][b][:k]) for b in range(len(q))]
            print(f"small_batch={sb} k={k} ok={ok}", flush=True)
            for b in range(len(q)):
                if not ok[b]:
                    print(f"   q{b} (row {q[b]}) ids {list(map(int, ids[b]))} gold {list(map(int, g['ids_nofilter'][b][:k]))}"
                          f" sc {list(np.round(sc[b], 6))} gold sc {list(np.round(g['scores_nofilter'][b][:k], 6))}",
                          flush=True)
    rows = idx.get_rows(np.arange(len(x)))
    print("rows finite", bool(np.isfinite(rows).all()), "norms", np.linalg.norm(rows, axis=1)[:4], flush=True)
    idx.close()


if __name__ == "__main__":
    main()
