"""MI355X: the device's draws use the host libm's exp / log bit for bit.

The reference's draws (code/neal8.cpp:95-102, code/split_merge.cpp:204-215) compare a
uniform against cumulative probabilities built from glibc's `exp`.  The device evaluates
those exps with glibc's algorithm and tables (csrc/glibc_math.hpp, `dexp` in
csrc/kernels.hip); the device libm (ocml) differs from glibc in the last ulp for some
inputs, and a uniform placed between the two cumulative values flips the draw.  These tests
(1) compare the device exp / log with the host libm on a grid, (2) construct log-weights
whose ocml and glibc exps differ with the uniform between the two boundaries -- the ocml
path draws differently from the reference, the engine's path does not -- and (3) place the
uniform exactly on every cumulative boundary of random weight vectors.
"""
import ctypes
import math

import numpy as np
import pytest

import pyref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import split_and_merge_gibbs_sampling_amd as hd
    hd.build()
    e = hd.Engine(0)
    yield e
    e.close()


class FixedU:
    """A stream that yields one given uniform (pyref.sample_prob1's rng argument)."""

    def __init__(self, u):
        self.u = u

    def unif(self):
        return self.u


def ref_draw(logw, rU):
    """n8:95-102 with the host libm: exp(probs - max), / sum, Rcpp sample(..., probs)."""
    mx = max(logw)
    p = [math.exp(v - mx) for v in logw]
    s = 0.0
    for x in p:
        s += x
    return pyref.sample_prob1(FixedU(rU), [x / s for x in p])


def ref_two_way(v0, v1, rU, expf=math.exp):
    """sm:204-215: the same draw over two entries (revsort of two: equal -> second first)."""
    mx = max(v0, v1)
    p0, p1 = expf(v0 - mx), expf(v1 - mx)
    s = p0 + p1
    p0, p1 = p0 / s, p1 / s
    s2 = (p0 if p0 > 0 else 0.0) + (p1 if p1 > 0 else 0.0)
    p0, p1 = p0 / s2, p1 / s2
    first0 = p0 > p1
    a0 = p0 if first0 else p1
    return (0 if first0 else 1) if rU <= a0 else (1 if first0 else 0)


def p0_of(e):
    """p0 of the two-entry draw with weights (1, e), in the reference's operation order."""
    s = 1.0 + e
    p0, p1 = 1.0 / s, e / s
    s2 = p0 + p1
    return p0 / s2


def grid():
    rng = np.random.default_rng(5)
    return np.concatenate([rng.uniform(-745.0, 0.0, 100_000), rng.uniform(-40.0, 0.0, 200_000),
                           -np.abs(rng.standard_normal(100_000)) * 1e-3,
                           np.array([0.0, -0.0, -np.inf, -1e-300, -708.5, -709.9, -744.9, -0.5, -1.0])])


def test_device_exp_log_are_host_libm(eng):
    x = grid()
    host = np.array([math.exp(v) for v in x])
    dev = eng.debug_math(x, "exp")
    assert np.array_equal(dev.view(np.uint64), host.view(np.uint64))
    y = np.concatenate([np.exp(x[np.isfinite(x)]), np.random.default_rng(6).uniform(1e-12, 1.0, 50_000)])
    y = y[y > 0]
    hl = np.array([math.log(v) for v in y])
    dl = eng.debug_math(y, "log")
    assert np.array_equal(dl.view(np.uint64), hl.view(np.uint64))


def test_device_log_of_counts_is_host_libm(eng):
    # log(n) of cluster sizes: the resolver and the restricted scan take it from the glibc
    # replica on the device where the host reads its logn table (std::log)
    y = np.concatenate([np.arange(1, 1 << 21, dtype=np.float64),
                        np.random.default_rng(7).uniform(1.0, 1e12, 100_000)])
    dl = eng.debug_math(y, "log")
    assert np.array_equal(dl.view(np.uint64), np.array([math.log(v) for v in y]).view(np.uint64))


def test_ulp_boundary_draws_follow_glibc(eng):
    x = grid()
    x = x[np.isfinite(x) & (x < -1e-6) & (x > -30.0)]
    host = np.array([math.exp(v) for v in x])
    ocml = eng.debug_math(x, "exp", ocml=True)
    differ = np.nonzero(ocml != host)[0]
    # the device libm does differ from glibc somewhere on the grid: the hole the replica closes
    assert differ.size > 0
    cases = 0
    for k in differ[:400]:
        pg, po = p0_of(host[k]), p0_of(ocml[k])
        if pg == po:
            continue              # the ulp was absorbed by the normalisation
        rU = max(pg, po)          # picks 0 under the larger p0, 1 under the smaller
        logw = [0.0, float(x[k])]
        want = ref_draw(logw, rU)
        assert want == ref_two_way(0.0, float(x[k]), rU)
        assert eng.debug_draw(logw, rU) == want
        assert eng.debug_draw(logw, rU, two_way=True) == want
        # the device libm's exp draws the other entry here
        assert eng.debug_draw(logw, rU, ocml=True) != want
        assert eng.debug_draw(logw, rU, two_way=True, ocml=True) != want
        cases += 1
        if cases >= 25:
            break
    assert cases > 0


@pytest.mark.parametrize("E", [2, 5, 23, 70])
def test_draw_on_every_cumulative_boundary(eng, E):
    rng = np.random.default_rng(100 + E)
    for trial in range(12):
        logw = list(rng.normal(0.0, 3.0, E))
        if trial % 3 == 1:
            logw[int(rng.integers(E))] = -math.inf       # an empty cluster (log 0)
        if trial % 3 == 2:
            logw[1] = logw[0]                            # a tie (revsort order)
        mx = max(logw)
        p = [math.exp(v - mx) for v in logw]
        s = 0.0
        for v in p:
            s += v
        p = [v / s for v in p]
        tot = 0.0
        for v in p:
            if v > 0:
                tot += v
        p = [v / tot for v in p]
        perm = list(range(1, E + 1))
        pyref.revsort(p, perm)
        cum, c = [], 0.0
        for v in p:
            c += v
            cum.append(c)
        for b in cum[:-1]:
            for rU in (b, math.nextafter(b, 1.0), math.nextafter(b, 0.0)):
                if not 0.0 < rU < 1.0:
                    continue
                assert eng.debug_draw(logw, rU) == ref_draw(logw, rU), (E, trial, rU)


# ------------------------------------------------------------------ Walker alias (> 200)
@pytest.mark.parametrize("E", [230, 256])
def test_walker_draws_match_reference(eng, E):
    """More than 200 entries with n p > 0.1: Rcpp's sample() uses Walker's alias method
    (R random.c walker_ProbSampleReplace); the device's n8 draw builds the same table."""
    rng = np.random.default_rng(E)
    for trial in range(10):
        logw = list(rng.normal(0.0, 0.3, E))
        if trial % 2:
            logw[0] += 3.0                          # one heavy entry
        p = np.exp(np.array(logw) - max(logw))
        assert (E * p / p.sum() > 0.1).sum() > 200  # the Walker branch of Rcpp sample()
        for rU in list(rng.random(20)) + [1e-9, 0.5, 1 - 1e-9]:
            assert eng.debug_draw(logw, float(rU)) == ref_draw(logw, float(rU)), (E, trial, rU)


def _walker_dataset():
    from split_and_merge_gibbs_sampling_amd.data import Dataset
    rng = np.random.default_rng(17)
    att = np.array([250, 4, 2, 3], np.int32)
    n = 480
    codes = np.stack([rng.integers(1, a + 1, size=n) for a in att], axis=1).astype(np.uint8)
    return Dataset(codes, att, np.full(4, 6.0), np.full(4, 0.25), 0.68, np.zeros(n, np.int32), "walker")


def test_walker_update_phi_center_draws(hd_mod, oracle):
    """update_phi's center draw over an attribute with m_j = 250 levels: a small cluster with
    a large sigma has near-flat level probabilities, so sample(1:m_j, 1, TRUE, prob)
    (cf:199) takes Walker's path on the host as in the reference."""
    ds = _walker_dataset()
    K = 160
    c = (np.arange(ds.n) % K).astype(np.int32)
    rng = np.random.default_rng(3)
    cen = np.stack([rng.integers(1, ds.attrisize + 1) for _ in range(K)]).astype(np.float64)
    sig = rng.uniform(2.0, 6.0, size=(K, ds.d))
    st = oracle.seed_state(12)
    e = hd_mod.Engine(0)
    e.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    e.set_state(c, cen, sig)
    e.rng_state = st
    ost = oracle.OracleState(c, K, cen, sig)
    for _ in range(3):
        e.update_phi()
        assert oracle.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, ost, st) == 0
        c2, cen2, sig2 = e.get_state()
        assert np.array_equal(cen2, ost.centers[:K]) and np.array_equal(sig2, ost.sigma[:K])
        assert np.array_equal(e.rng_state, st)
    e.close()


@pytest.mark.parametrize("K", [240, 480])
def test_walker_neal8_sweeps(hd_mod, oracle, K):
    """Neal-8 draws over K + m > 200 comparable entries (n8:99-102 -> Walker): K = 240
    exercises the register path of the device draw, K = 480 (every point its own cluster)
    the LDS path."""
    ds = _walker_dataset()
    c = (np.arange(ds.n) % K).astype(np.int32)
    rng = np.random.default_rng(4)
    cen = np.stack([rng.integers(1, ds.attrisize + 1) for _ in range(K)]).astype(np.float64)
    sig = rng.uniform(3.0, 8.0, size=(K, ds.d))
    st = oracle.seed_state(13)
    pc, ps, _ = oracle.pool_generate(ds.attrisize, ds.v, ds.w, ds.n * 3, st)
    e = hd_mod.Engine(0)
    e.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    e.set_state(c, cen, sig)
    e.set_pool(pc, ps)
    e.rng_state = st
    ost = oracle.OracleState(c, K, cen, sig)
    for _ in range(2):
        e.neal8_sweep(3)
        assert oracle.neal8_sweep(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, ost, 3, pc, ps, st, fast=1) == 0
        c2, cen2, sig2 = e.get_state()
        assert cen2.shape[0] == ost.K and np.array_equal(c2, ost.c_i)
        assert np.array_equal(cen2, ost.centers[:ost.K]) and np.array_equal(sig2, ost.sigma[:ost.K])
        assert np.array_equal(e.rng_state, st)
    e.close()


@pytest.fixture(scope="module")
def hd_mod():
    import split_and_merge_gibbs_sampling_amd as hd
    hd.build()
    return hd
