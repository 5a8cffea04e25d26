"""qnorm.h's qn_elem: (float)(x / nrm) from a per-row reciprocal, dividing only near an f32
rounding boundary.  The same IEEE f64 operations in numpy over random rows and adversarial
near-boundary quotients: the result always equals the f64 division rounded to f32."""
import numpy as np


def qn_elem(x, nrm):
    rinv = 1.0 / nrm
    q = x * rinv
    e = np.abs(q) * 2.0 ** -50
    lo, hi = (q - e).astype(np.float32), (q + e).astype(np.float32)
    exact = (x / nrm).astype(np.float32)
    return np.where(lo == hi, lo, exact), lo == hi


def test_random_rows_match_division():
    rng = np.random.default_rng(0)
    n = 2_000_000
    x = rng.standard_normal(n).astype(np.float32).astype(np.float64) * 10.0 ** rng.integers(-6, 6, n)
    nrm = np.sqrt(rng.random(n) * 1e3 + 1e-3)
    got, fast = qn_elem(x, nrm)
    assert np.array_equal(got.view(np.uint32), (x / nrm).astype(np.float32).view(np.uint32))
    assert fast.mean() > 0.999  # the division is the rare path


def test_near_boundary_quotients():
    """Quotients placed on / next to f32 midpoints: the fast path must not decide those."""
    rng = np.random.default_rng(1)
    f = rng.standard_normal(200_000).astype(np.float32)
    mid = (f.astype(np.float64) + np.nextafter(f, np.float32(np.inf)).astype(np.float64)) / 2
    nrm = 1.0 + rng.random(200_000)
    for k in (-3, -1, 0, 1, 3):
        target = mid * (1 + k * 2.0 ** -52)
        x = (target * nrm).astype(np.float32).astype(np.float64)  # an f32 element, as the kernels see
        got, _ = qn_elem(x, nrm)
        assert np.array_equal(got.view(np.uint32), (x / nrm).astype(np.float32).view(np.uint32))
    x = mid * nrm  # (an f64 x: the quotient right at a midpoint)
    got, fast = qn_elem(x, nrm)
    assert np.array_equal(got.view(np.uint32), (x / nrm).astype(np.float32).view(np.uint32))
    assert not fast.all()
