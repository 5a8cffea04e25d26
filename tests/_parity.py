"""Near-tie-gated list comparison shared by the GPU parity tests.

The bar (north_star): top-K index sets bit-exact on identical fp32 inputs, scores within
1e-5.  The reference ranks in fp32 BLAS, whose summation order differs from any other
implementation by ~1e-7, so where two candidates are closer than GAP the id order between
them is not determined by the reference either.  A query is "gated" when the K-th and
(K+1)-th reference scores are closer than GAP: its scores are still checked, and its id set
must still hold every reference item scoring more than GAP above the K-th; only the items
tied with the boundary within GAP may differ.  Every test reports how many queries were gated
(`Gate.report`) and asserts a ceiling on it, so a silently widening gate shows up.
"""
import os

import numpy as np

TOL = 1e-5
GAP = 2e-6

# every Gate.report of the session; tests/conftest.py writes them to gpurun_out/parity_gates.json
# at the end of the run (a -q run prints nothing, the file keeps the counts)
RECORDS = []


class Gate:
    def __init__(self, name):
        self.name = name
        self.checked = 0
        self.gated = 0

    def report(self, max_frac):
        n = self.checked + self.gated
        print(f"[parity] {self.name}: {self.checked} queries id-checked, {self.gated} near-tie gated "
              f"(K-th/(K+1)-th reference gap < {GAP:g}) of {n}")
        RECORDS.append({"gate": self.name, "test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0],
                        "queries": n, "id_checked": self.checked, "near_tie_gated": self.gated,
                        "max_gated_frac": max_frac})
        assert self.gated <= max_frac * n, (self.name, self.gated, n)
        return self.gated


def check_row(gate, sc, ids, ref_ids, ref_sc, k, ref_next=None, order=True, tol=TOL):
    """One query: device (sc, ids) against the reference top list (ref_ids, ref_sc), which
    may be shorter than k (fewer eligible items); ref_next is the (k+1)-th reference score,
    or None when there is none.  Empty device slots must hold id -1."""
    ref_ids = np.asarray(ref_ids)
    ref_sc = np.asarray(ref_sc, np.float64)
    L = len(ref_ids)
    assert L <= k
    assert np.all(np.asarray(ids[L:]) == -1), ids[L:]
    np.testing.assert_allclose(np.asarray(sc[:L], np.float64), ref_sc, atol=tol, rtol=0)
    boundary_open = ref_next is None or L < k or (ref_sc[L - 1] - ref_next) > GAP
    if not boundary_open:
        # only the near-tied boundary items may differ: every reference item clearly above
        # the boundary must still be in the device list
        gate.gated += 1
        sure = set(int(i) for i, s in zip(ref_ids, ref_sc) if s > ref_sc[L - 1] + GAP)
        assert sure <= set(int(i) for i in ids[:L]), (sorted(sure - set(int(i) for i in ids[:L])))
        return False
    gate.checked += 1
    assert set(int(i) for i in ids[:L]) == set(int(i) for i in ref_ids), (ids[:L], ref_ids)
    if order and L > 1 and np.all(-np.diff(ref_sc) > GAP):
        assert list(ids[:L]) == list(ref_ids)
    return True


def blend_sure(c_ids, c_sc, f_ids, f_sc, ks, wc, wf, k):
    """Items of the hybrid's final top-k (union blend of the two sides' top-ks lists,
    recommendation_system.py:789-843) that do NOT depend on a near-tied side boundary, with
    their blended scores.  c_* / f_*: each side's reference list sorted descending, longer than
    ks (the items around the boundary).  A side item is certainly in its top-ks list when it
    scores more than GAP above the ks-th, certainly out when more than GAP below; in between
    its membership is open.  An item whose memberships are all certain has a fixed blend h; it
    is certainly in the final top-k when fewer than k other items can reach h - GAP with every
    open membership chosen in their favour.  Returns {item: h}."""
    def sides(ids, sc):
        ids, sc = list(ids), np.asarray(sc, np.float64)
        if len(ids) <= ks:
            return {int(i): (1, s) for i, s in zip(ids, sc)}   # every eligible item is in
        b = sc[ks - 1]
        return {int(i): ((1 if s > b + GAP else 0 if s < b - GAP else None), s) for i, s in zip(ids, sc)}
    C, F = sides(c_ids, c_sc), sides(f_ids, f_sc)
    items = set(C) | set(F)
    h_fix, h_max = {}, {}
    for i in items:
        mc, sc_ = C.get(i, (0, 0.0))
        mf, sf_ = F.get(i, (0, 0.0))
        if mc == 0 and mf == 0:
            continue
        opts_c = [0.0, wc * sc_] if mc is None else [wc * sc_ * mc]
        opts_f = [0.0, wf * sf_] if mf is None else [wf * sf_ * mf]
        h_max[i] = max(a + b for a in opts_c for b in opts_f)
        if mc is not None and mf is not None:
            h_fix[i] = wc * sc_ * mc + wf * sf_ * mf
    sure = {}
    for i, h in h_fix.items():
        rivals = sum(1 for j, hm in h_max.items() if j != i and hm >= h - GAP)
        if rivals < k:
            sure[i] = h
    return sure
