"""Edge shapes on the MI355X: chains of 1-200 points against the CPU oracle.

These are the shapes the reference handles and round 2 failed on:
a sweep whose LAST point opens a cluster (case 3 / case 4 of n8:107-159) skipped the
device's sweep-end kernels, so the labels stayed slot ids and the carried frequency tables
missed the sweep's moves -- wrong log-likelihoods at N = 4, an E_GSL at N = 7, a host heap
fault in split-merge at N = 2 (labels >= K indexed the host state) and an E_VALIDATE on a
one-attribute chain.  Every shape runs Neal-8 only, split-merge only, and both, with the
move log active at every N (no recount threshold), through run_markov_chain (la:6-174) and
through the pipelined iteration API (hdpm_iterations, the path bench.py times).

Labels, K and the 625-word R stream must be identical to the oracle's after every saved
iteration; log-likelihoods within 1e-10 relative (north_star).  When the oracle's chain
stops with an error (validate_state / norm_const2 throw), the engine must stop with the
same status.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-10

# (n, d, k, levels): k ground-truth clusters, levels = m_j (or a (lo, hi) range)
TINY = [(1, 1, 1, 2), (2, 1, 1, 2), (2, 3, 2, 3), (3, 2, 2, 2), (4, 3, 2, 3), (7, 5, 3, 4), (7, 3, 2, 3),
        (16, 3, 2, 3), (33, 3, 2, 3), (64, 3, 2, 3), (65, 1, 2, 3), (100, 1, 1, 2), (130, 3, 4, (2, 5)),
        (200, 3, 2, 3)]
MODES = {"n8": (True, False), "sm": (False, True), "both": (True, True)}


@pytest.fixture(scope="module")
def hd():
    import split_and_merge_gibbs_sampling_amd as hd
    hd.build()
    return hd


def _data(shape):
    from split_and_merge_gibbs_sampling_amd.data import hamming_mixture
    n, d, k, levels = shape
    return hamming_mixture(n, d, k, levels, seed=40 + n + d)


def _oracle_chain(oracle, ds, iters, m, n8, sm, seed, L=1, c_i="truth"):
    ci = ds.truth if c_i == "truth" else c_i
    rng = oracle.seed_state(seed)
    st, ref = oracle.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, m=m, iterations=iters, L=L,
                                      c_i=ci, burnin=0, neal8=n8, split_merge=sm, rng=rng, fast=1)
    return st, ref, rng


def _shape_id(s):
    return "x".join(str(v).replace(" ", "") for v in s)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("m", [1, 3])
@pytest.mark.parametrize("shape", TINY, ids=_shape_id)
def test_tiny_shapes_chain_matches_oracle(hd, oracle, shape, m, mode):
    n8, sm = MODES[mode]
    if sm and shape[0] < 2:
        pytest.skip("split-merge draws two distinct points (sm:278): N >= 2")
    ds = _data(shape)
    iters = 8
    st, ref, rng = _oracle_chain(oracle, ds, iters, m, n8, sm, seed=5)
    kw = dict(m=m, iterations=iters, L=1, c_i=ds.truth, burnin=0, neal8=n8, split_merge=sm)
    if st != 0:
        with pytest.raises(hd.HdpmError) as ex:
            hd.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=5, **kw)
        assert ex.value.status == st
        return
    res = hd.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=5, **kw)
    assert np.array_equal(res["total_cls"], ref["total_cls"])
    assert np.array_equal(res["c_i"], ref["c_i"])
    assert np.array_equal(res["accepted"], ref["accepted"])
    np.testing.assert_allclose(res["loglikelihood"], ref["loglikelihood"], rtol=RTOL, atol=0)
    assert np.array_equal(res["rng_state"], rng)


# debug 33554432 (bit 25): the fixed-point resolver (k_resolve_fp) for every launch, not only
# after a launch that listed >= 64 points
# debug 33554432 | 1073741824 (bits 25, 30): the device-wide fixed-point resolver (k_resolve_fpg,
# a workgroup per 512-point chunk, grid barriers) for every launch
@pytest.mark.parametrize("debug", [0, 33554432, 33554432 | 1073741824])
@pytest.mark.parametrize("mode", ["n8", "both"])
@pytest.mark.parametrize("shape", [(2, 1, 1, 2), (4, 3, 2, 3), (7, 5, 3, 4), (65, 1, 2, 3), (130, 3, 4, (2, 5))],
                         ids=_shape_id)
def test_tiny_shapes_iteration_api(hd, oracle, shape, mode, debug):
    # hdpm_iterations (prepared next sweep launched ahead, speculative update_phi, carried
    # tables) in batches of uneven length; state and stream compared after every batch
    n8, sm = MODES[mode]
    ds = _data(shape)
    m = 3
    batches = [1, 4, 7]
    iters = sum(batches)
    st, ref, _ = _oracle_chain(oracle, ds, iters, m, n8, sm, seed=9)
    e = hd.Engine(0)
    try:
        e.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
        e.set_seed(9)
        e.set_debug(debug)
        e.init_chain(e.chain_params(m=m, iterations=iters, L=1, burnin=0, neal8=n8, split_merge=sm), c_i=ds.truth)
        it = 0
        for b in batches:
            try:
                _, ll = e.iterations(it, b)
            except hd.HdpmError as ex:
                assert st != 0 and ex.status == st
                return
            for q in range(b):
                np.testing.assert_allclose(ll[q], ref["loglikelihood"][it + q], rtol=RTOL, atol=0)
            it += b
            c, cen, _ = e.get_state()
            assert cen.shape[0] == ref["total_cls"][it - 1]
            assert np.array_equal(c, ref["c_i"][it - 1])
        assert st == 0
    finally:
        e.close()


@pytest.mark.parametrize("debug", [0, 16, 33554432, 33554432 | 1073741824])
def test_tiny_shape_random_init_chain(hd, oracle, debug):
    # random L = 5 initial labels on 40 points: clusters vanish (case 2) and appear (cases 3 /
    # 4) within the same sweeps, at the last point too; carried tables (0), recounts (16), the
    # fixed-point resolver for every launch (33554432)
    ds = _data((40, 4, 3, 3))
    iters = 12
    for seed in range(1, 40):
        st, ref, rng = _oracle_chain(oracle, ds, iters, 2, True, True, seed=seed, L=5, c_i=None)
        if st == 0:
            break
    assert st == 0
    e = hd.Engine(0)
    try:
        e.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
        e.set_seed(seed)
        e.set_debug(debug)
        res = e.run_markov_chain(m=2, iterations=iters, L=5, c_i=None, burnin=0, neal8=True, split_merge=True)
        assert np.array_equal(res["c_i"], ref["c_i"])
        np.testing.assert_allclose(res["loglikelihood"], ref["loglikelihood"], rtol=RTOL, atol=0)
        assert np.array_equal(e.rng_state, rng)
    finally:
        e.close()
