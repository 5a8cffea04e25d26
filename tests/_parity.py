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
import numpy as np

TOL = 1e-5
GAP = 2e-6


class Gate:
    def __init__(self, name):
        self.name = name
        self.checked = 0
        self.gated = 0

    def report(self, max_frac):
        n = self.checked + self.gated
        print(f"[parity] {self.name}: {self.checked} queries id-checked, {self.gated} near-tie gated "
              f"(K-th/(K+1)-th reference gap < {GAP:g}) of {n}")
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
