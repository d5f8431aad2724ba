"""Host-side posterior summaries of the reference script (zoo_simulator.R:193-236):
mcclust::arandi and LaplacesDemon::ESS / IAT restated in posterior.py.  The R packages are
absent (parity unpinned); arandi is pinned to scikit-learn's adjusted Rand score, ESS and
IAT to the closed forms of an AR(1) chain."""
import numpy as np
import pytest

from split_and_merge_gibbs_sampling_amd import posterior as P


def test_arandi_matches_sklearn():
    sk = pytest.importorskip("sklearn.metrics")
    rng = np.random.default_rng(1)
    for n, k1, k2 in [(50, 3, 4), (500, 7, 7), (2000, 20, 5)]:
        a = rng.integers(0, k1, n)
        b = np.where(rng.random(n) < 0.7, a % k2, rng.integers(0, k2, n))
        assert abs(P.arandi(a, b) - sk.adjusted_rand_score(a, b)) < 1e-12
    a = rng.integers(0, 5, 100)
    assert P.arandi(a, a) == pytest.approx(1.0)
    assert P.arandi(a, (a + 1) % 5) == pytest.approx(1.0)     # label-invariant


def ar1(n, rho, seed):
    rng = np.random.default_rng(seed)
    x = np.zeros(n)
    e = rng.standard_normal(n)
    for t in range(1, n):
        x[t] = rho * x[t - 1] + e[t]
    return x


def test_ess_iid_and_ar1():
    n = 20000
    iid = np.random.default_rng(2).standard_normal(n)
    assert 0.85 * n <= P.ess(iid)[0] <= n
    rho = 0.8
    e = P.ess(np.stack([ar1(n, rho, 3), iid], 1))
    assert e[0] == pytest.approx(n * (1 - rho) / (1 + rho), rel=0.2)
    assert P.ess(np.ones(100))[0] == 1.0                      # constant chain


def test_iat_ar1():
    rho = 0.8
    assert P.iat(ar1(50000, rho, 4)) == pytest.approx((1 + rho) / (1 - rho), rel=0.25)
    assert P.iat(np.random.default_rng(5).standard_normal(20000)) == pytest.approx(1.0, abs=0.2)
