"""MI355X parity tests: the HIP path through the C ABI against the CPU oracle and the
committed golden traces.  Integer results (labels, K, Hamming counts) and the per-point
log-likelihood matrix must be bit-exact; reductions (compute_loglikelihood,
logprobgs_c_i) are compared with a relative tolerance of 1e-10 (north_star)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
RTOL = 1e-10


@pytest.fixture(scope="module")
def hd():
    import split_and_merge_gibbs_sampling_amd as hd
    hd.build()
    return hd


def make_engine(hd, ds):
    e = hd.Engine(0)
    e.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    return e


def random_params(ds, K, seed):
    rng = np.random.default_rng(seed)
    cen = np.stack([rng.integers(1, ds.attrisize + 1) for _ in range(K)]).astype(np.float64)
    sig = rng.uniform(0.15, 2.5, size=(K, ds.d))
    return cen, sig


def synth(n, d, k, levels, seed=1):
    from split_and_merge_gibbs_sampling_amd.data import hamming_mixture
    return hamming_mixture(n, d, k, levels, seed=seed)


def oracle_state(oracle, c, cen, sig):
    return oracle.OracleState(c, cen.shape[0], cen, sig)


def assert_same_state(eng, ost):
    c, cen, sig = eng.get_state()
    assert cen.shape[0] == ost.K
    assert np.array_equal(c, ost.c_i)
    assert np.array_equal(cen, ost.centers[:ost.K])
    assert np.array_equal(sig, ost.sigma[:ost.K])


# ------------------------------------------------------------------ loglik matrix
@pytest.mark.parametrize("which", ["zoo", "synth32", "synth200"])
def test_loglik_matrix_bit_exact(hd, oracle, zoo, which):
    ds = {"zoo": zoo, "synth32": synth(3000, 32, 7, 2), "synth200": synth(700, 200, 5, (2, 6))}[which]
    K = 9
    cen, sig = random_params(ds, K, 1)
    c = np.arange(ds.n, dtype=np.int32) % K
    eng = make_engine(hd, ds)
    eng.set_state(c, cen, sig)
    L, H = eng.loglik_matrix(K)
    Lo, Ho = oracle.loglik_matrix(ds.codes, ds.attrisize, cen, sig)
    assert np.array_equal(H, Ho)
    assert np.array_equal(L, Lo)          # bit-exact: same tables, same j order
    eng.close()


# ------------------------------------------------------------------ single sweep
def sweep_case(hd, oracle, ds, c, cen, sig, P, seed, m=3, debug=0, sweeps=1, phi=False, phi_device=False):
    st = oracle.seed_state(seed)
    pc, ps, s0 = oracle.pool_generate(ds.attrisize, ds.v, ds.w, P, st)
    assert s0 == 0
    eng = make_engine(hd, ds)
    eng.set_debug(debug)
    if phi_device:
        eng.set_phi_device(True, general=phi_device == "general")
    eng.set_state(c, cen, sig)
    eng.set_pool(pc, ps)
    eng.rng_state = st
    ost = oracle_state(oracle, c, cen, sig)
    ost_rng = st.copy()
    for it in range(sweeps):
        eng.neal8_sweep(m)
        r = oracle.neal8_sweep(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, ost, m, pc, ps, ost_rng, fast=1)
        assert r == 0
        assert_same_state(eng, ost)
        assert np.array_equal(eng.rng_state, ost_rng), f"rng diverged after sweep {it}"
        if phi:
            eng.update_phi()
            assert oracle.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, ost, ost_rng) == 0
            assert_same_state(eng, ost)
            assert np.array_equal(eng.rng_state, ost_rng)
    stats = eng.stats()
    eng.close()
    return stats


# debug 0: default (snapshot speculation in the exact-rows kernel), 1: every point on the
# exact path in the resolver, 8: no speculation (the resolver decides every listed point)
# 8192: the resolver's block mode for every launch (parallel decisions, serial walk)
@pytest.mark.parametrize("debug", [0, 1, 8, 2048, 8192])
def test_zoo_single_sweeps_from_truth(hd, oracle, zoo, debug):
    cen, sig = random_params(zoo, 7, 3)
    stats = sweep_case(hd, oracle, zoo, zoo.truth, cen, sig, zoo.n * 3, seed=17, debug=debug, sweeps=3)
    assert stats["sweeps"] == 3


def test_zoo_sweeps_with_update_phi_all_singletons(hd, oracle, zoo):
    # L = 101 (every point its own cluster): exercises cases 2 and 4 heavily
    c = np.arange(zoo.n, dtype=np.int32)
    cen, sig = random_params(zoo, zoo.n, 5)
    sweep_case(hd, oracle, zoo, c, cen, sig, zoo.n * 3, seed=23, sweeps=4, phi=True)


@pytest.mark.parametrize("debug", [0, 8, 8192])
def test_zoo_sweeps_with_update_phi_one_cluster(hd, oracle, zoo, debug):
    # L = 1: the first sweeps create clusters (case 3 -> device restarts)
    c = np.zeros(zoo.n, np.int32)
    cen, sig = random_params(zoo, 1, 6)
    stats = sweep_case(hd, oracle, zoo, c, cen, sig, zoo.n * 3, seed=29, sweeps=6, phi=True, debug=debug)
    assert stats["restarts"] > 0


# 16: recount the frequency tables every update_phi; 128: no speculative update_phi;
# 2048: exact rows one wave per point; 4096: no block mode in the resolver; 8192: block mode
# for every launch
@pytest.mark.parametrize("phi_device", [False, True])
@pytest.mark.parametrize("debug", [0, 1, 8, 16, 128, 2048, 2048 | 1, 4096, 8192, 8192 | 8, 262144])
def test_synthetic_sweeps_with_update_phi(hd, oracle, debug, phi_device):
    ds = synth(6000, 32, 8, 2, seed=3)
    cen, sig = random_params(ds, 8, 7)
    sweep_case(hd, oracle, ds, ds.truth, cen, sig, ds.n * 3, seed=31, sweeps=3, phi=True, debug=debug,
               phi_device=phi_device)


def test_speculative_update_phi(hd, oracle):
    # Separated clusters from the truth: after the first update_phi the sweeps move few or no
    # points, so update_phi comes (entirely, or for a prefix of labels) from the pass the host
    # ran during the sweep; every step is compared with the oracle.
    ds = synth(4000, 64, 6, 4, seed=9)
    cen, sig = random_params(ds, 6, 11)
    stats = sweep_case(hd, oracle, ds, ds.truth, cen, sig, ds.n * 3, seed=41, sweeps=8, phi=True, debug=524288)
    assert stats["phi_spec_runs"] >= 6
    assert stats["phi_spec_clusters"] > 0


# update_phi on the device (csrc/phi.hip): centers, sigmas, tables and the stream position
# after it against the oracle, on shapes with one and several attribute classes, binary and
# many-level attributes, wide rows; and that the device path ran (no silent host fallback).
# path: "fast" (launch_phi2, the default where every pick is fixed), "trees" (the general
# kernels' composition trees), "walks" (debug bit 27: the per-start-drift walks, k_phi_cwalk)
@pytest.mark.parametrize("path", ["fast", "trees", "walks"])
@pytest.mark.parametrize("shape", ["c5_like", "mixed", "binary", "wide", "zoo"])
def test_device_update_phi(hd, oracle, zoo, shape, path):
    if shape == "zoo":
        ds, K = zoo, 7
    else:
        ds, K = {"c5_like": (synth(8000, 128, 12, 4, seed=5), 12), "mixed": (synth(5000, 48, 9, (2, 6), seed=6), 9),
                 "binary": (synth(6000, 32, 8, 2, seed=7), 8), "wide": (synth(2500, 784, 6, 6, seed=8), 6)}[shape]
    cen, sig = random_params(ds, K, 13)
    stats = sweep_case(hd, oracle, ds, ds.truth, cen, sig, ds.n * 3, seed=43, sweeps=4, phi=True,
                       phi_device=True if path == "fast" else "general", debug=134217728 if path == "walks" else 0)
    phis = {k: v for k, v in stats.items() if "phi" in k}
    assert stats["phi_device_calls"] >= 2, phis
    if path == "fast":
        # (random parameters: some picks depend on the uniform, and such updates are handed to
        # the general kernels; test_device_update_phi_fast_path_converged covers commits)
        if shape in ("c5_like", "mixed", "wide"):
            assert stats["phi_fast_calls"] >= 1, phis
    elif path == "walks":
        assert stats["phi_tree_calls"] == 0 and stats["phi_fast_calls"] == 0, stats
    elif shape != "wide":
        # d <= 128: the composition trees resolve the drifts, a cluster with a pick that
        # depends on the uniform by the walks inside the same update (no re-run)
        assert stats["phi_tree_calls"] >= 2 and stats["phi_tree_retries"] == 0, \
            {k: v for k, v in stats.items() if "phi" in k}


def converged_params(ds, c, K, sigma=0.5):
    """Centers at each cluster's per-attribute mode, sigmas `sigma`: the state of a converged
    chain (every update_phi center pick fixed by its cluster's frequency table)."""
    cen = np.zeros((K, ds.d))
    for k in range(K):
        rows = ds.codes[c == k]
        for j in range(ds.d):
            cen[k, j] = np.bincount(rows[:, j], minlength=int(ds.attrisize[j]) + 1)[1:].argmax() + 1
    return cen, np.full((K, ds.d), sigma)


# The fast path (launch_phi2) from a converged state: every update commits there (no hand-back
# to the general kernels), C5-, C3- and C4-like shapes, the chain bit-identical to the oracle.
@pytest.mark.parametrize("shape", ["c5_like", "c3_like", "c4_like", "binary"])
def test_device_update_phi_fast_path_converged(hd, oracle, shape):
    ds, K = {"c5_like": (synth(20000, 128, 10, 4, seed=15), 10), "c3_like": (synth(12000, 64, 8, (2, 6), seed=16), 8),
             "c4_like": (synth(6000, 784, 5, 6, seed=17), 5), "binary": (synth(8000, 32, 6, 2, seed=18), 6)}[shape]
    cen, sig = converged_params(ds, ds.truth, K)
    stats = sweep_case(hd, oracle, ds, ds.truth, cen, sig, ds.n * 3, seed=44, sweeps=5, phi=True, phi_device=True)
    phis = {k: v for k, v in stats.items() if "phi" in k}
    # (a speculation beside a sweep that then moved points is dropped and the update re-run)
    assert stats["phi_fast_calls"] >= 5 and stats["phi_fast_handbacks"] == 0, phis
    assert stats["phi_device_calls"] == 5, phis


def test_device_update_phi_small_clusters_fall_back_or_match(hd, oracle, zoo):
    # all-singleton Zoo clusters: rhig's bisection path and center levels that depend on the
    # uniform; whatever the device hands back, the chain is the oracle's
    c = np.arange(zoo.n, dtype=np.int32)
    cen, sig = random_params(zoo, zoo.n, 5)
    stats = sweep_case(hd, oracle, zoo, c, cen, sig, zoo.n * 3, seed=23, sweeps=3, phi=True, phi_device=True)
    assert stats["phi_device_calls"] + stats["phi_device_fallbacks"] == 3


def test_device_update_phi_subset_then_loglik(hd, oracle):
    # a full device update_phi sums the regrouped log-likelihood and caches it; a following
    # update_phi of a label subset (device or host) changes parameters without a label change,
    # so compute_loglikelihood must not return the cached sum
    ds = synth(8000, 64, 6, (2, 5), seed=12)
    cen, sig = random_params(ds, 6, 14)
    st = oracle.seed_state(47)
    pc, ps, _ = oracle.pool_generate(ds.attrisize, ds.v, ds.w, ds.n * 3, st)
    eng = make_engine(hd, ds)
    eng.set_phi_device(True)
    eng.set_state(ds.truth, cen, sig)
    eng.set_pool(pc, ps)
    eng.rng_state = st
    ost = oracle_state(oracle, ds.truth, cen, sig)
    rng = st.copy()
    for it in range(2):
        eng.neal8_sweep(3)
        assert oracle.neal8_sweep(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, ost, 3, pc, ps, rng, fast=1) == 0
        eng.update_phi()
        assert oracle.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, ost, rng) == 0
        ll = eng.compute_loglikelihood()
        ref = oracle.compute_loglikelihood(ds.codes, ds.attrisize, ost)
        assert abs(ll - ref) <= RTOL * abs(ref)
        sub = [0, 2] if it == 0 else [1]
        eng.update_phi(sub)
        assert oracle.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, ost, rng, idx=sub) == 0
        assert_same_state(eng, ost)
        assert np.array_equal(eng.rng_state, rng)
        ll = eng.compute_loglikelihood()
        ref = oracle.compute_loglikelihood(ds.codes, ds.attrisize, ost)
        assert abs(ll - ref) <= RTOL * abs(ref), f"stale log-likelihood after a subset update ({it})"
    assert eng.stats()["phi_device_calls"] >= 2
    eng.close()


def test_synthetic_large_d_sweep(hd, oracle):
    ds = synth(1500, 300, 4, (2, 6), seed=4)
    cen, sig = random_params(ds, 4, 8)
    sweep_case(hd, oracle, ds, ds.truth, cen, sig, ds.n * 3, seed=37, sweeps=2, phi=True)


# ------------------------------------------------------------------ loglikelihood
def test_compute_loglikelihood_matches_sequential_sum(hd, oracle, zoo):
    for ds in (zoo, synth(20000, 64, 10, (2, 6), seed=5)):
        cen, sig = random_params(ds, 10, 9)
        c = (np.arange(ds.n) % 10).astype(np.int32)
        eng = make_engine(hd, ds)
        eng.set_state(c, cen, sig)
        got = eng.compute_loglikelihood()
        ref = oracle.compute_loglikelihood(ds.codes, ds.attrisize, oracle_state(oracle, c, cen, sig))
        assert abs(got - ref) <= RTOL * abs(ref)
        eng.close()


def test_compute_loglikelihood_from_counts_after_update_phi(hd, oracle):
    # after a sweep + update_phi the engine regroups the sum into per-(cluster, attribute)
    # match counts; it must agree with the per-point kernel (debug bit 2) and the oracle
    ds = synth(30000, 96, 6, (2, 5), seed=8)
    cen, sig = random_params(ds, 6, 11)
    eng = make_engine(hd, ds)
    eng.set_seed(5)
    eng.set_state(ds.truth, cen, sig)
    eng.generate_pool(ds.n * 2)
    for _ in range(2):
        eng.neal8_sweep(2)
        eng.update_phi()
        fast = eng.compute_loglikelihood()
        eng.set_debug(4)
        slow = eng.compute_loglikelihood()
        eng.set_debug(0)
        c, cen2, sig2 = eng.get_state()
        ref = oracle.compute_loglikelihood(ds.codes, ds.attrisize, oracle_state(oracle, c, cen2, sig2))
        assert abs(fast - slow) <= 1e-12 * abs(slow)
        assert abs(fast - ref) <= RTOL * abs(ref)
    eng.close()


# ------------------------------------------------------------------ split-merge pieces
def test_restricted_gibbs_matches_oracle(hd, oracle, zoo):
    cen, sig = random_params(zoo, 7, 10)
    c = zoo.truth.astype(np.int32).copy()
    i1, i2 = 3, 50
    S = [i for i in range(zoo.n) if i not in (i1, i2) and c[i] in (c[i1], c[i2])]
    st = oracle.seed_state(41)
    eng = make_engine(hd, zoo)
    eng.set_state(c, cen, sig)
    eng.rng_state = st
    eng.restricted_gibbs(S, i1, i2, t=5)
    ost = oracle_state(oracle, c, cen, sig)
    assert oracle.restricted_gibbs(zoo.codes, zoo.attrisize, zoo.v, zoo.w, S, ost, i1, i2, 5, st) == 0
    assert_same_state(eng, ost)
    assert np.array_equal(eng.rng_state, st)
    eng.close()


def test_restricted_gibbs_large_clusters(hd, oracle):
    ds = synth(8000, 32, 4, 2, seed=6)
    cen, sig = random_params(ds, 4, 11)
    c = ds.truth.astype(np.int32).copy()
    i1 = int(np.where(c == 1)[0][0])
    i2 = int(np.where(c == 2)[0][0])
    S = [i for i in range(ds.n) if i not in (i1, i2) and c[i] in (c[i1], c[i2])]
    st = oracle.seed_state(43)
    eng = make_engine(hd, ds)
    eng.set_state(c, cen, sig)
    eng.rng_state = st
    eng.restricted_gibbs(S, i1, i2, t=3)
    ost = oracle_state(oracle, c, cen, sig)
    assert oracle.restricted_gibbs(ds.codes, ds.attrisize, ds.v, ds.w, S, ost, i1, i2, 3, st) == 0
    assert_same_state(eng, ost)
    eng.close()


# d >= 128: the scans' update_phi goes through the engine's pipelined update_phi job
# (split_merge.inl hupdate_phi_job); debug 128 keeps the one-pass path
@pytest.mark.parametrize("debug", [0, 128])
def test_restricted_gibbs_wide_update_phi(hd, oracle, debug):
    ds = synth(3000, 200, 4, 6, seed=39)
    cen, sig = random_params(ds, 4, 12)
    c = ds.truth.astype(np.int32).copy()
    i1 = int(np.where(c == 2)[0][0])
    i2 = int(np.where(c == 1)[0][0])              # c1 > c2: update_phi in ascending label order
    S = [i for i in range(ds.n) if i not in (i1, i2) and c[i] in (c[i1], c[i2])]
    st = oracle.seed_state(44)
    eng = make_engine(hd, ds)
    eng.set_debug(debug)
    eng.set_state(c, cen, sig)
    eng.rng_state = st
    eng.restricted_gibbs(S, i1, i2, t=4)
    ost = oracle_state(oracle, c, cen, sig)
    assert oracle.restricted_gibbs(ds.codes, ds.attrisize, ds.v, ds.w, S, ost, i1, i2, 4, st) == 0
    assert_same_state(eng, ost)
    assert np.array_equal(eng.rng_state, st)
    eng.close()


def test_run_markov_chain_wide_split_merge_matches_oracle(hd, oracle):
    ds = synth(1200, 160, 4, 5, seed=40)
    kw = dict(m=3, iterations=8, L=4, burnin=2, t=3, r=3, neal8=True, split_merge=True)
    st, ref = oracle.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=17, fast=1, **kw)
    assert st == 0
    res = hd.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=17, **kw)
    assert np.array_equal(res["c_i"], ref["c_i"])
    assert np.array_equal(res["total_cls"], ref["total_cls"])


def test_logprobgs_c_i_matches_oracle(hd, oracle, zoo):
    cen, sig = random_params(zoo, 7, 12)
    c = zoo.truth.astype(np.int32).copy()
    i1, i2 = 0, 60
    S = [i for i in range(zoo.n) if i not in (i1, i2) and c[i] in (c[i1], c[i2])]
    g = c.copy()
    rng = np.random.default_rng(1)
    for s in S:
        g[s] = c[i1] if rng.random() < 0.5 else c[i2]
    eng = make_engine(hd, zoo)
    eng.set_state(c, cen, sig)
    got = eng.logprobgs_c_i(g, S, i1, i2)
    ref = oracle.logprobgs_c_i(zoo.codes, zoo.attrisize, oracle_state(oracle, c, cen, sig), g, S, i1, i2)
    assert abs(got - ref) <= RTOL * max(1.0, abs(ref))
    eng.close()


# ------------------------------------------------------------------ full chains vs golden
def test_run_markov_chain_zoo_neal8_golden(hd, zoo):
    g = np.load(os.path.join(G, "zoo_neal8_seed1.npz"))
    res = hd.run_markov_chain(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w, m=3, iterations=40, L=1,
                              c_i=np.zeros(zoo.n, np.int32), burnin=0, neal8=True, split_merge=False, seed=1)
    assert np.array_equal(res["c_i"], g["c_i"])
    assert np.array_equal(res["total_cls"], g["total_cls"])
    np.testing.assert_allclose(res["loglikelihood"], g["loglikelihood"], rtol=RTOL, atol=0)


def test_run_markov_chain_zoo_split_merge_golden(hd, zoo):
    g = np.load(os.path.join(G, "zoo_sm_seed7.npz"))
    res = hd.run_markov_chain(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w, m=3, iterations=30, L=1,
                              c_i=np.zeros(zoo.n, np.int32), burnin=0, t=10, r=10, neal8=True, split_merge=True,
                              seed=7)
    assert np.array_equal(res["c_i"], g["c_i"])
    assert np.array_equal(res["accepted"], g["accepted"])
    np.testing.assert_allclose(res["loglikelihood"], g["loglikelihood"], rtol=RTOL, atol=0)


def test_run_markov_chain_keep_params_and_stream_handback(hd, oracle, zoo):
    """The adapter's contract: centers / sigmas of every saved iteration
    (la:144-147), and the random stream handed back so that a second chain started from it
    continues the reference's stream (consecutive R calls without set.seed)."""
    kw = dict(m=3, iterations=12, L=1, c_i=np.zeros(zoo.n, np.int32), burnin=3, t=10, r=10, neal8=True,
              split_merge=True)
    a = hd.run_markov_chain(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w, seed=7, **kw)
    b = hd.run_markov_chain(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w, seed=7, keep_params=True, **kw)
    for k in ("c_i", "total_cls", "accepted", "final_ass"):
        assert np.array_equal(a[k], b[k]), k
    np.testing.assert_allclose(a["loglikelihood"], b["loglikelihood"], rtol=RTOL, atol=0)
    assert len(b["centers"]) == 12
    for it in range(12):
        assert b["centers"][it].shape == (b["total_cls"][it], zoo.d) == b["sigmas"][it].shape
    st = oracle.seed_state(7)
    ost, ref = oracle.run_markov_chain(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w, rng=st, fast=1, **kw)
    assert ost == 0 and np.array_equal(ref["c_i"], b["c_i"])
    assert np.array_equal(b["rng_state"], st) and np.array_equal(a["rng_state"], st)
    c = hd.run_markov_chain(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w, rng_state=b["rng_state"], **kw)
    ost, ref2 = oracle.run_markov_chain(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w, rng=st, fast=1, **kw)
    assert ost == 0 and np.array_equal(ref2["c_i"], c["c_i"]) and np.array_equal(c["rng_state"], st)


@pytest.mark.parametrize("shape", ["settled", "moving"])
def test_iterations_record_matches_stepwise(hd, oracle, shape):
    """hdpm_iterations_record (the adapter's sampling loop, la:139-153, thinning 1 and 2): every
    saved iteration's K, labels, centers and sigmas equal what hdpm_iteration + hdpm_get_state
    give step by step, the labels equal the oracle's chain; the labels come from the host mirror
    (the sweep's move log applied) rather than N-word downloads once the chain settles."""
    ds = synth(20000, 64, 8, 4, seed=71) if shape == "settled" else synth(6000, 32, 6, 2, seed=72)
    for thinning in (1, 2):
        iters, burnin = 12, 2
        kw = dict(m=3, iterations=iters, L=1, c_i=ds.truth, burnin=burnin, neal8=True, split_merge=False,
                  thinning=thinning)
        st, ref = oracle.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=8, fast=1, **kw)
        assert st == 0
        a = make_engine(hd, ds)
        a.set_seed(8)
        p = a.chain_params(m=3, iterations=iters, L=1, burnin=burnin, neal8=True, split_merge=False, thinning=thinning)
        a.init_chain(p, c_i=ds.truth)
        total = (iters + burnin) * thinning
        acc, ll, kk, cis, cens, sigs = a.iterations_record(0, 5)
        acc2, ll2, kk2, cis2, cens2, sigs2 = a.iterations_record(5, total - 5)
        kk, cis = np.concatenate([kk, kk2]), np.concatenate([cis, cis2])
        cens, sigs, ll = cens + cens2, sigs + sigs2, np.concatenate([ll, ll2])
        stats = a.stats()
        a.close()
        assert len(kk) == iters and np.array_equal(cis, ref["c_i"]) and np.array_equal(kk, ref["total_cls"])
        b = make_engine(hd, ds)
        b.set_seed(8)
        b.init_chain(p, c_i=ds.truth)
        q = 0
        for it in range(total):
            _, lik = b.iteration(it)
            assert lik == ll[it]
            if it >= thinning * burnin and it % thinning == 0:
                c, cen, sig = b.get_state()
                assert np.array_equal(c, cis[q]) and np.array_equal(cen, cens[q]) and np.array_equal(sig, sigs[q])
                q += 1
        b.close()
        assert q == iters
        if shape == "settled":
            assert stats["labels_downloaded"] <= 2, stats


def test_run_markov_chain_random_init_matches_oracle(hd, oracle, zoo):
    # L = 20 random labels, a seed whose initial draw uses all 20 labels
    seed = next(s for s in range(1, 100)
                if len(np.unique((20 * oracle.runif(oracle.seed_state(s), zoo.n) + 1).astype(int))) == 20)
    kw = dict(m=3, iterations=15, L=20, burnin=5, t=4, r=4, neal8=True, split_merge=True)
    st, ref = oracle.run_markov_chain(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w, seed=seed, fast=1, **kw)
    assert st == 0
    res = hd.run_markov_chain(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w, seed=seed, **kw)
    assert np.array_equal(res["c_i"], ref["c_i"])
    assert np.array_equal(res["total_cls"], ref["total_cls"])


def test_run_markov_chain_unused_label_is_an_error(hd, oracle, zoo):
    seed = next(s for s in range(1, 100)
                if len(np.unique((20 * oracle.runif(oracle.seed_state(s), zoo.n) + 1).astype(int))) < 20)
    with pytest.raises(hd.HdpmError) as e:
        hd.run_markov_chain(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w, m=3, iterations=2, L=20,
                            burnin=0, neal8=True, split_merge=False, seed=seed)
    assert e.value.status == 1


def test_synthetic_chain_matches_oracle(hd, oracle):
    ds = synth(10000, 32, 20, 2, seed=10091995)
    kw = dict(m=3, iterations=3, L=1, c_i=ds.truth, burnin=0, neal8=True, split_merge=False)
    st, ref = oracle.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=2, fast=1, **kw)
    assert st == 0
    res = hd.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=2, **kw)
    assert np.array_equal(res["c_i"], ref["c_i"])
    np.testing.assert_allclose(res["loglikelihood"], ref["loglikelihood"], rtol=RTOL, atol=0)


def test_iteration_api_prepared_sweeps(hd, oracle):
    # hdpm_iteration prepares the next sweep (draws reserved, update_phi speculated on the
    # host pool); reading the stream state or the labels in between cancels it, which must
    # leave no trace: labels and log-likelihoods follow the oracle's chain either way.
    ds = synth(5000, 64, 8, 4, seed=12)
    iters = 8
    kw = dict(m=3, iterations=iters, L=1, c_i=ds.truth, burnin=0, neal8=True, split_merge=False)
    st, ref = oracle.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=4, fast=1, **kw)
    assert st == 0
    eng = make_engine(hd, ds)
    eng.set_seed(4)
    params = eng.chain_params(m=3, iterations=iters, L=1, burnin=0, neal8=True, split_merge=False)
    eng.init_chain(params, c_i=ds.truth)
    for it in range(iters):
        _, ll = eng.iteration(it)
        assert abs(ll - ref["loglikelihood"][it]) <= RTOL * abs(ref["loglikelihood"][it])
        if it % 3 == 1:
            c, _, _ = eng.get_state()
            assert np.array_equal(c, ref["c_i"][it])
        if it % 3 == 2:
            _ = eng.rng_state
    c, _, _ = eng.get_state()
    assert np.array_equal(c, ref["c_i"][iters - 1])
    stats = eng.stats()
    assert stats["phi_spec_clusters"] > 0
    eng.close()
    # the batch API launches each next sweep before the host has finished the iteration
    eng = make_engine(hd, ds)
    eng.set_seed(4)
    eng.init_chain(params, c_i=ds.truth)
    _, ll = eng.iterations(0, 5)
    np.testing.assert_allclose(ll, ref["loglikelihood"][:5], rtol=RTOL, atol=0)
    _, ll = eng.iterations(5, iters - 5)
    np.testing.assert_allclose(ll, ref["loglikelihood"][5:], rtol=RTOL, atol=0)
    c, _, _ = eng.get_state()
    assert np.array_equal(c, ref["c_i"][iters - 1])
    eng.close()


# ------------------------------------------------------------------ size-independent properties
def test_large_sweep_invariants(hd):
    from split_and_merge_gibbs_sampling_amd.data import config
    ds = config("c5", n=200_000)
    eng = make_engine(hd, ds)
    eng.set_seed(5)
    K = 20
    cen, sig = random_params(ds, K, 13)
    eng.set_state(ds.truth, cen, sig)
    eng.update_phi()
    eng.generate_pool(ds.n * 3)
    for _ in range(2):
        eng.neal8_sweep(3)
        eng.update_phi()
    c, cen, sig = eng.get_state()
    K = cen.shape[0]
    assert set(np.unique(c)) == set(range(K))          # labels contiguous, none empty
    assert np.all(sig > 0) and np.all(cen >= 1) and np.all(cen <= ds.attrisize)
    ll = eng.compute_loglikelihood()
    assert np.isfinite(ll) and ll < 0
    eng.close()


# ------------------------------------------------------------------ device random stream
@pytest.mark.parametrize("pre", [0, 1, 623, 624, 1000, 5000])
def test_device_mt_stream_matches_r(hd, oracle, zoo, pre):
    eng = make_engine(hd, zoo)
    st = oracle.seed_state(77)
    oracle.runif(st, pre)                      # start mid-block
    eng.rng_state = st
    for count in (1, 623, 624, 625, 20000):
        got = eng.rng_fill_device(count)
        ref = oracle.runif(st, count)
        u = got.astype(np.float64) * 2.3283064365386963e-10
        assert np.array_equal(u, ref)           # no 0 draws in these ranges: fixup inactive
        assert np.array_equal(eng.rng_state, st)
    eng.close()


@pytest.mark.parametrize("pre", [0, 311, 624])
def test_device_mt_stream_jump_ahead_matches_r(hd, oracle, zoo, pre):
    # windows of at least 256 * 624 * 8 draws use 256 workgroups started by jump polynomials
    eng = make_engine(hd, zoo)
    st = oracle.seed_state(2718)
    oracle.runif(st, pre)
    eng.rng_state = st
    for count in (400_000, 1_300_001, 2_500_000):
        got = eng.rng_fill_device(count)
        ref = oracle.runif(st, count)
        assert np.array_equal(got.astype(np.float64) * 2.3283064365386963e-10, ref)
        assert np.array_equal(eng.rng_state, st)
    eng.close()


# ------------------------------------------------------------------ latent pool generator
def _pool_case(hd, oracle, ds, v, w, P, pre, seed, debug=0):
    eng = hd.Engine(0)
    eng.set_data(ds.codes, ds.attrisize, ds.gamma, v, w)
    eng.set_debug(debug)
    st = oracle.seed_state(seed)
    oracle.runif(st, pre)
    eng.rng_state = st
    eng.generate_pool(P)
    pc, ps, _ = oracle.pool_generate(ds.attrisize, v, w, P, st)
    gc, gs = eng.get_pool(P)
    assert np.array_equal(gc, pc)
    assert np.array_equal(gs, ps)                 # bit-exact sigmas
    assert np.array_equal(eng.rng_state, st)      # same stream position after the pool
    stats = eng.stats()
    eng.close()
    return stats


@pytest.mark.parametrize("pre", [0, 1, 623, 624, 5000])
def test_device_pool_matches_oracle_zoo(hd, oracle, zoo, pre):
    st = _pool_case(hd, oracle, zoo, zoo.v, zoo.w, 303, pre, 31 + pre)
    assert st["pool_device_calls"] == 1


# c5_large: 200k entries (~1,560 chunks / 25 groups of the segment parse, k_pool_seg*); serial_parse: debug
# bit 28, the entry starts by the sequential host walk over the device's acceptance tables
@pytest.mark.parametrize("case", ["mixed_levels", "odd_d_bc", "c5_like", "c5_large", "serial_parse", "host_forced"])
def test_device_pool_matches_oracle_synthetic(hd, oracle, case):
    if case == "mixed_levels":
        ds = synth(2000, 64, 5, (2, 6), seed=3)
        v, w, P = np.full(64, 6.0), np.full(64, 0.25), 6000
    elif case == "odd_d_bc":
        ds = synth(1500, 7, 4, (2, 7), seed=4)
        v = np.array([1.8, 1.8, 6.0, 6.0, 3.0, 1.5, 6.0])      # v - 1 < 1: rbeta algorithm BC
        w = np.array([0.25, 0.25, 0.25, 0.4, 0.5, 0.3, 0.25])
        P = 4500
    else:
        ds = synth(3000, 128, 6, 4, seed=5)
        v, w, P = np.full(128, 6.0), np.full(128, 0.25), 30000   # ~14M draws: multi-workgroup slice
        if case == "c5_large":
            P = 200_000
    debug = {"host_forced": 64, "serial_parse": 268435456}.get(case, 0)
    st = _pool_case(hd, oracle, ds, v, w, P, 77, 9, debug=debug)
    assert st["pool_device_calls"] == (0 if case == "host_forced" else 1)
    if case != "host_forced":
        # the segment parse's chain stayed in its windows (no serial fallback) unless forced
        assert st["pool_walk_fallbacks"] == (1 if case == "serial_parse" else 0), \
            {k: st[k] for k in ("pool_walk_fallbacks", "pool_device_calls", "t_pool_parse_ms")}


def test_device_pool_then_sweeps_match_oracle(hd, oracle):
    # the prepass / exact rows read the device-built pool records and tables
    ds = synth(4000, 96, 6, (2, 5), seed=12)
    cen, sig = random_params(ds, 6, 3)
    eng = make_engine(hd, ds)
    st = oracle.seed_state(5)
    eng.rng_state = st
    eng.set_state(ds.truth, cen, sig)
    P = ds.n * 3
    eng.generate_pool(P)
    ost = oracle_state(oracle, ds.truth.astype(np.int32).copy(), cen.copy(), sig.copy())
    pc, ps, _ = oracle.pool_generate(ds.attrisize, ds.v, ds.w, P, st)
    for _ in range(3):
        eng.neal8_sweep(3)
        oracle.neal8_sweep(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, ost, 3, pc, ps, st)
        assert_same_state(eng, ost)
        eng.update_phi()
        oracle.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, ost, st)
        assert_same_state(eng, ost)
    assert eng.stats()["pool_device_calls"] == 1
    eng.close()


# ------------------------------------------------------------------ pool-entry heads
def _head_bound_check(oracle, ds, heads, pc, ps, npts=600, nent=400, seed=0):
    """Every head bound (csrc/kernels.hpp 'Pool-entry heads') is >= the entry's exact row
    value for sampled points: A_up - max(dmin H, S_a + (H - h_a) dmin, S_b + (H - h_b) dmin),
    and the head's codes, dmin and partial sums are those of the entry."""
    rng = np.random.default_rng(seed)
    pts = rng.choice(ds.n, size=min(npts, ds.n), replace=False)
    ents = rng.choice(pc.shape[0], size=min(nent, pc.shape[0]), replace=False)
    L, _ = oracle.loglik_matrix(ds.codes[pts], ds.attrisize, pc[ents], ps[ents])     # exact rows
    d = ds.d
    mmax = int(ds.attrisize.max())
    wb = 1 if mmax <= 2 else 2 if mmax <= 4 else 4 if mmax <= 16 else 8
    wd = -(-d // 64)
    Ws = 2 if wd <= 2 else 4 if wd <= 4 else wd           # kernels.hpp plane_words
    hw = wb * Ws + 2
    assert heads.shape[1] >= hw and np.all(heads[:, hw:] == 0)
    heads = heads[:, :hw]
    q = 1.0 / ds.attrisize
    mu, sd = (1 - q).sum(), np.sqrt(((1 - q) * q).sum())
    ha, hb = max(0, int(np.floor(mu - 4 * sd))), max(0, int(np.floor(mu - 1.25 * sd)))
    h = heads[ents]
    bits = lambda wds: np.array([[(int(w[j >> 6]) >> (j & 63)) & 1 for j in range(d)] for w in wds])  # noqa: E731
    code = sum(bits(h[:, b * Ws:(b + 1) * Ws]) << b for b in range(wb)) + 1
    assert np.array_equal(code, pc[ents].astype(np.int64))
    f32 = lambda w: (w & 0xffffffff).astype(np.uint32).view(np.float32).astype(np.float64)  # noqa: E731
    A_up, dmin = f32(h[:, -2]), f32(h[:, -2] >> 32)
    Sa, Sb = f32(h[:, -1]), f32(h[:, -1] >> 32)
    e = np.exp(1.0 / ps[ents])
    den = np.log(1.0 + (ds.attrisize - 1.0) / e)
    dd = (-den) - (-1.0 / ps[ents] - den)
    srt = np.sort(dd, 1)
    assert np.all(dmin <= srt[:, 0]) and np.all(dmin >= srt[:, 0] * (1 - 1e-6))
    for S, hh in ((Sa, ha), (Sb, hb)):
        ref = srt[:, :hh].sum(1)
        assert np.all(S <= ref) and np.all(S >= ref * (1 - 1e-6) - 1e-30)
    M = ds.codes[pts][:, None, :] != pc[ents][None, :, :]      # npts x nent x d
    H = M.sum(-1)
    low = dmin[None] * H
    low = np.maximum(low, np.where(H >= ha, Sa[None] + (H - ha) * dmin[None], 0))
    low = np.maximum(low, np.where(H >= hb, Sb[None] + (H - hb) * dmin[None], 0))
    ub = A_up[None] - low
    assert np.all(ub >= L), float((L - ub).max())
    return float(np.median(ub - L))


@pytest.mark.parametrize("src", ["device", "host"])
def test_pool_heads_bound_exact_rows(hd, oracle, src):
    ds = synth(3000, 128, 6, 4, seed=21)
    eng = make_engine(hd, ds)
    st = oracle.seed_state(13)
    eng.rng_state = st
    P = 9000
    if src == "device":
        eng.generate_pool(P)
        pc, ps = eng.get_pool(P)
    else:
        pc, ps, _ = oracle.pool_generate(ds.attrisize, ds.v, ds.w, P, st)
        eng.set_pool(pc, ps)
    heads = eng.get_pool_heads(P)
    _head_bound_check(oracle, ds, heads, pc, ps)
    eng.close()


def test_pool_heads_binary_and_absent(hd, oracle):
    ds = synth(2000, 32, 6, 2, seed=22)                # wb = 1: codes and scalars in 4 words
    eng = make_engine(hd, ds)
    st = oracle.seed_state(14)
    pc, ps, _ = oracle.pool_generate(ds.attrisize, ds.v, ds.w, 6000, st)
    eng.set_pool(pc, ps)
    _head_bound_check(oracle, ds, eng.get_pool_heads(6000), pc, ps)
    eng.close()
    wide = synth(500, 200, 4, (2, 6), seed=23)         # d = 200, m_j <= 6: Ws = 4, wb = 4 (18 words)
    eng = make_engine(hd, wide)
    pc, ps, _ = oracle.pool_generate(wide.attrisize, wide.v, wide.w, 1500, st)
    eng.set_pool(pc, ps)
    _head_bound_check(oracle, wide, eng.get_pool_heads(1500), pc, ps, npts=300, nent=300)
    eng.close()
    wider = synth(300, 300, 4, 4, seed=26)             # d = 300: Ws = 5, wb = 2, wide prepass heads
    eng = make_engine(hd, wider)
    pc, ps, _ = oracle.pool_generate(wider.attrisize, wider.v, wider.w, 900, st)
    eng.set_pool(pc, ps)
    heads = eng.get_pool_heads(900)
    assert heads.shape[1] == 16                        # 12 words padded to a multiple of 8
    _head_bound_check(oracle, wider, heads, pc, ps, npts=200, nent=200)
    eng.close()
    c4ish = synth(200, 784, 4, 6, seed=29)             # C4's layout: Ws = 13, wb = 4, 56-word heads
    eng = make_engine(hd, c4ish)
    pc, ps, _ = oracle.pool_generate(c4ish.attrisize, c4ish.v, c4ish.w, 600, st)
    eng.set_pool(pc, ps)
    heads = eng.get_pool_heads(600)
    assert heads.shape[1] == 56
    _head_bound_check(oracle, c4ish, heads, pc, ps, npts=100, nent=150)
    eng.close()
    widest = synth(100, 2100, 3, 2, seed=30)           # Ws = 33 > 32: generic prepass, no heads
    eng = make_engine(hd, widest)
    pc, ps, _ = oracle.pool_generate(widest.attrisize, widest.v, widest.w, 300, st)
    eng.set_pool(pc, ps)
    with pytest.raises(hd.HdpmError):
        eng.get_pool_heads(300)
    eng.close()


# 1024: full bound records for the latent picks (no heads) on a head-eligible layout
@pytest.mark.parametrize("debug", [0, 1024, 8192])
def test_c5_like_sweeps_heads_and_records(hd, oracle, debug):
    ds = synth(5000, 128, 8, 4, seed=24)
    cen, sig = random_params(ds, 8, 25)
    sweep_case(hd, oracle, ds, ds.truth, cen, sig, ds.n * 3, seed=43, sweeps=3, phi=True, debug=debug)


@pytest.mark.parametrize("debug", [0, 1024])
def test_wide_mixed_levels_sweeps_heads_and_records(hd, oracle, debug):
    ds = synth(3000, 200, 6, (2, 6), seed=27)          # Ws = 4, wb = 4 heads
    cen, sig = random_params(ds, 6, 28)
    sweep_case(hd, oracle, ds, ds.truth, cen, sig, ds.n * 3, seed=47, sweeps=3, phi=True, debug=debug)


# k_prepass_wide (16-lane group per point) against the oracle on wide layouts, with heads,
# with full records (1024) and with the generic one-thread-per-point prepass (16384).  The
# chain starts from the ground truth with update_phi'd parameters (hdpm_init_chain), so
# most points are certified by the bounds and the rest take exact rows.
@pytest.mark.parametrize("debug", [0, 1024, 16384])
@pytest.mark.parametrize("shape", ["c4", "c4_k80", "ws18_binary", "ws5_wb8", "ws5_wb2", "ws20_wb2", "ws16_wb4"])
def test_wide_prepass_sweeps(hd, oracle, debug, shape):
    if shape == "c4":
        ds = synth(4000, 784, 6, 6, seed=31)           # Ws = 13, wb = 4 (C4's layout)
    elif shape == "c4_k80":
        ds = synth(4000, 784, 80, 6, seed=36)          # cluster summaries beyond the LDS budget
    elif shape == "ws18_binary":
        ds = synth(3000, 1100, 5, 2, seed=32)          # Ws = 18: two plane words per lane
    elif shape == "ws5_wb8":
        ds = synth(2000, 300, 5, 20, seed=33)          # Ws = 5, wb = 8
    elif shape == "ws5_wb2":
        ds = synth(2000, 300, 5, 4, seed=37)           # Ws = 5, wb = 2
    elif shape == "ws20_wb2":
        ds = synth(2000, 1250, 5, 4, seed=38)          # Ws = 20, wb = 2: two words per lane
    else:
        ds = synth(1500, 1024, 5, 6, seed=39)          # Ws = 16, wb = 4: wb Ws = 64, the widest heads (66 words)
    eng = make_engine(hd, ds)
    eng.set_seed(35)
    eng.set_debug(debug)
    params = eng.chain_params(m=3, iterations=1, L=0, burnin=0, neal8=True, split_merge=False)
    eng.init_chain(params, c_i=ds.truth)
    c, cen, sig = eng.get_state()
    pc, ps = eng.get_pool(ds.n * 3)
    ost = oracle_state(oracle, c.copy(), cen.copy(), sig.copy())
    st = eng.rng_state.copy()
    for _ in range(3):
        eng.neal8_sweep(3)
        assert oracle.neal8_sweep(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, ost, 3, pc, ps, st) == 0
        assert_same_state(eng, ost)
        assert np.array_equal(eng.rng_state, st)
        eng.update_phi()
        assert oracle.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, ost, st) == 0
        assert_same_state(eng, ost)
        assert np.array_equal(eng.rng_state, st)
    stats = eng.stats()
    if debug == 0:
        assert stats["listed_points"] < 3 * ds.n // 2, stats     # the bounds certify most points
    eng.close()


def test_hig_logspace_chain_large_clusters(hd, oracle):
    # Two clusters of ~1.5k members: the SM priors' 2F1 series (hg:11-48) overflows, so the
    # reference throws (HDPM_E_GSL).  With the HDPM_OPT_HIG_LOGSPACE extension the chain
    # runs and follows the oracle's mirror of the extension step for step.
    ds = synth(3000, 16, 2, 2, seed=3)
    kw = dict(m=3, iterations=10, L=1, c_i=ds.truth, burnin=0, t=3, r=3, neal8=True, split_merge=True)
    with pytest.raises(hd.HdpmError) as e:
        hd.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=5, **kw)
    assert e.value.status == 2
    try:
        oracle.set_hig_logspace(True)
        st, ref = oracle.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=5, fast=1, **kw)
    finally:
        oracle.set_hig_logspace(False)
    assert st == 0
    res = hd.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=5, hig_logspace=True, **kw)
    assert np.array_equal(res["c_i"], ref["c_i"])
    assert np.array_equal(res["total_cls"], ref["total_cls"])
    assert np.array_equal(res["accepted"], ref["accepted"])
    np.testing.assert_allclose(res["loglikelihood"], ref["loglikelihood"], rtol=RTOL, atol=0)


# Moves over |S| >= 4096 points: the scans draw from the device windows (debug bit 16 keeps
# them on the host); wide rows (d = 160) also take the pipelined update_phi job.
@pytest.mark.parametrize("debug", [0, 65536])
def test_split_merge_chain_large_moves(hd, oracle, debug):
    ds = synth(10000, 160, 2, 3, seed=42)
    kw = dict(m=3, iterations=6, L=1, c_i=ds.truth, burnin=0, t=3, r=3, neal8=True, split_merge=True)
    try:
        oracle.set_hig_logspace(True)
        st, ref = oracle.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=6, fast=2, **kw)
    finally:
        oracle.set_hig_logspace(False)
    assert st == 0
    eng = make_engine(hd, ds)
    try:
        eng.set_hig_logspace(True)
        eng.set_seed(6)
        eng.set_debug(debug)
        res = eng.run_markov_chain(**kw)
        assert eng.stats()["sm_moves"] == 6
    finally:
        eng.close()
    assert np.array_equal(res["c_i"], ref["c_i"])
    assert np.array_equal(res["total_cls"], ref["total_cls"])
    assert np.array_equal(res["accepted"], ref["accepted"])
    np.testing.assert_allclose(res["loglikelihood"], ref["loglikelihood"], rtol=RTOL, atol=0)


@pytest.mark.parametrize("wait_us", [None, 0])
def test_split_merge_chain_wide_scan_and_give_up(hd, oracle, wait_us):
    """Split-merge moves whose restricted scans (|S| >= 512) walk on many CUs
    (k_sm_scan_wide), and with a zero barrier limit give up at once and walk on one workgroup:
    the same chain as the oracle either way."""
    ds = synth(6000, 64, 2, 3, seed=44)
    kw = dict(m=3, iterations=4, L=1, c_i=ds.truth, burnin=0, t=3, r=3, neal8=True, split_merge=True)
    try:
        oracle.set_hig_logspace(True)
        st, ref = oracle.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=8, fast=2, **kw)
    finally:
        oracle.set_hig_logspace(False)
    assert st == 0
    eng = make_engine(hd, ds)
    try:
        eng.set_hig_logspace(True)
        eng.set_seed(8)
        if wait_us is not None:
            eng.set_sm_wide_wait_us(wait_us)
        res = eng.run_markov_chain(**kw)
        stats = eng.stats()
    finally:
        eng.close()
    assert np.array_equal(res["c_i"], ref["c_i"])
    assert np.array_equal(res["total_cls"], ref["total_cls"])
    assert np.array_equal(res["accepted"], ref["accepted"])
    np.testing.assert_allclose(res["loglikelihood"], ref["loglikelihood"], rtol=RTOL, atol=0)
    assert stats["sm_wide_scans"] > 0, stats
    if wait_us == 0:
        assert stats["sm_wide_fallbacks"] == stats["sm_wide_scans"], stats
    else:
        assert stats["sm_wide_fallbacks"] == 0, stats


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4, 8, 9, 10])
def test_split_merge_device_chain(hd, oracle, mode):
    """The restricted Gibbs samplers of split-merge moves as one device chain (sm_chain: the t
    scans and their update_phi({c1, c2}) enqueued together, sm:163-225), scan by scan (mode 0),
    and chains stopped at scan k / its first / its second one-cluster update for k = 0, 2 (modes
    2-4, 8-10: the host continues from there): the same chain as the oracle every time."""
    ds = synth(6000, 64, 2, 3, seed=44)
    kw = dict(m=3, iterations=4, L=1, c_i=ds.truth, burnin=0, t=4, r=4, neal8=True, split_merge=True)
    try:
        oracle.set_hig_logspace(True)
        st, ref = oracle.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=8, fast=2, **kw)
    finally:
        oracle.set_hig_logspace(False)
    assert st == 0
    eng = make_engine(hd, ds)
    try:
        eng.set_hig_logspace(True)
        eng.set_seed(8)
        eng.set_sm_chain(mode)
        res = eng.run_markov_chain(**kw)
        stats = eng.stats()
    finally:
        eng.close()
    assert np.array_equal(res["c_i"], ref["c_i"])
    assert np.array_equal(res["total_cls"], ref["total_cls"])
    assert np.array_equal(res["accepted"], ref["accepted"])
    np.testing.assert_allclose(res["loglikelihood"], ref["loglikelihood"], rtol=RTOL, atol=0)
    if mode == 0:
        assert stats["sm_chain_runs"] == 0, stats
    else:
        assert stats["sm_chain_runs"] > 0, stats
        if mode >= 2:
            assert stats["sm_chain_resumes"] == stats["sm_chain_runs"], stats


def test_split_merge_second_dataset_other_attrisize(hd, oracle):
    """One engine, two data sets with the same d, v and w but other attribute sizes m_j: the
    split-merge priors' normalising constants norm_const2(w_j, v_j, m_j) (sm:419-436) must
    follow the new m_j (the cache was keyed on v / w only)."""
    kw = dict(m=3, iterations=4, L=1, burnin=0, t=3, r=3, neal8=True, split_merge=True)
    da = synth(900, 16, 3, 2, seed=61)
    db = synth(900, 16, 3, 5, seed=62)
    assert np.array_equal(da.v, db.v) and np.array_equal(da.w, db.w)
    eng = make_engine(hd, da)
    try:
        eng.set_seed(9)
        eng.run_markov_chain(c_i=da.truth, **kw)
        assert eng.stats()["sm_moves"] > 0
        eng.set_data(db.codes, db.attrisize, db.gamma, db.v, db.w)
        eng.set_seed(10)
        res = eng.run_markov_chain(c_i=db.truth, **kw)
    finally:
        eng.close()
    st, ref = oracle.run_markov_chain(db.codes, db.attrisize, db.gamma, db.v, db.w, seed=10, c_i=db.truth,
                                      fast=1, **kw)
    assert st == 0
    assert np.array_equal(res["c_i"], ref["c_i"])
    assert np.array_equal(res["accepted"], ref["accepted"])
    np.testing.assert_allclose(res["loglikelihood"], ref["loglikelihood"], rtol=RTOL, atol=0)


def test_restricted_gibbs_random_split_of_one_cluster(hd, oracle):
    # The split proposal's launch state: one true cluster's members dealt at random to two
    # labels with fresh parameters, so most scan draws are close calls whose pick depends
    # on the running sizes (k_sm_scan's interval test and its serial walk both run).
    ds = synth(9000, 24, 3, 2, seed=8)
    c = ds.truth.astype(np.int32).copy()
    K = 4
    members = np.where(c == 0)[0]
    rng = np.random.default_rng(5)
    c[members[rng.random(len(members)) < 0.5]] = 3
    i1 = int(members[c[members] == 0][0])
    i2 = int(members[c[members] == 3][0])
    cen, sig = random_params(ds, K, 13)
    S = [i for i in range(ds.n) if i not in (i1, i2) and c[i] in (c[i1], c[i2])]
    st = oracle.seed_state(47)
    eng = make_engine(hd, ds)
    eng.set_state(c, cen, sig)
    eng.rng_state = st
    eng.restricted_gibbs(S, i1, i2, t=6)
    ost = oracle_state(oracle, c, cen, sig)
    assert oracle.restricted_gibbs(ds.codes, ds.attrisize, ds.v, ds.w, S, ost, i1, i2, 6, st) == 0
    assert_same_state(eng, ost)
    assert np.array_equal(eng.rng_state, st)
    eng.close()


# |S| = 24k: several staged chunks of the scan; the draws come from the device generator
# windows (|S| >= 4096), or from the host stream (debug bit 16)
@pytest.mark.parametrize("debug", [0, 65536])
def test_restricted_gibbs_sizes_beyond_lds_logn(hd, oracle, debug):
    ds = synth(24000, 12, 2, 2, seed=9)
    c = ds.truth.astype(np.int32).copy()
    rng = np.random.default_rng(2)
    c[rng.random(ds.n) < 0.5] = 0
    c[c != 0] = 1
    i1 = int(np.where(c == 0)[0][0])
    i2 = int(np.where(c == 1)[0][0])
    cen, sig = random_params(ds, 2, 17)
    S = [i for i in range(ds.n) if i not in (i1, i2)]
    st = oracle.seed_state(53)
    eng = make_engine(hd, ds)
    eng.set_debug(debug)
    eng.set_state(c, cen, sig)
    eng.rng_state = st
    eng.restricted_gibbs(S, i1, i2, t=2)
    ost = oracle_state(oracle, c, cen, sig)
    assert oracle.restricted_gibbs(ds.codes, ds.attrisize, ds.v, ds.w, S, ost, i1, i2, 2, st) == 0
    assert_same_state(eng, ost)
    assert np.array_equal(eng.rng_state, st)
    eng.close()


# wide rows and a large S: device-window draws for the scans, then the pipelined update_phi
# job fed from the window's prefetched slice (Ctx::fill_stream_from)
@pytest.mark.parametrize("debug", [0, 65536])
def test_restricted_gibbs_wide_large_device_draws(hd, oracle, debug):
    ds = synth(9000, 160, 2, 4, seed=41)
    c = ds.truth.astype(np.int32).copy()
    i1 = int(np.where(c == 0)[0][0])
    i2 = int(np.where(c == 1)[0][0])
    cen, sig = random_params(ds, 2, 18)
    S = [i for i in range(ds.n) if i not in (i1, i2)]
    st = oracle.seed_state(55)
    eng = make_engine(hd, ds)
    eng.set_debug(debug)
    eng.set_state(c, cen, sig)
    eng.rng_state = st
    eng.restricted_gibbs(S, i1, i2, t=3)
    ost = oracle_state(oracle, c, cen, sig)
    assert oracle.restricted_gibbs(ds.codes, ds.attrisize, ds.v, ds.w, S, ost, i1, i2, 3, st) == 0
    assert_same_state(eng, ost)
    assert np.array_equal(eng.rng_state, st)
    eng.close()


def test_replica_chains_per_rank_seeds(hd, oracle):
    # bench.py --gpus N runs one chain per rank with seed 1 + rank (bench.rank_setup) on a
    # shared data set.  Two engines alive at once on one device, stepped
    # in alternation, must each follow the oracle's chain for their own seed: no state, stream
    # or host-pool slot shared between replicas.
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    ds = synth(4000, 32, 6, 3, seed=21)
    iters = 6
    kw = dict(m=3, iterations=iters, L=1, c_i=ds.truth, burnin=0, neal8=True, split_merge=False)
    seeds = [bench.rank_setup(r, 0)["seed"] for r in range(2)]
    assert seeds == [1, 2]
    refs = []
    for s in seeds:
        st, ref = oracle.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=s, fast=1, **kw)
        assert st == 0
        refs.append(ref)
    assert not np.array_equal(refs[0]["loglikelihood"], refs[1]["loglikelihood"])
    engs = []
    for s in seeds:
        e = make_engine(hd, ds)
        e.set_seed(s)
        e.init_chain(e.chain_params(m=3, iterations=iters, L=1, burnin=0, neal8=True, split_merge=False),
                     c_i=ds.truth)
        engs.append(e)
    for it in range(iters):
        for e, ref in zip(engs, refs):
            _, ll = e.iteration(it)
            assert abs(ll - ref["loglikelihood"][it]) <= RTOL * abs(ref["loglikelihood"][it])
    for e, ref in zip(engs, refs):
        c, _, _ = e.get_state()
        assert np.array_equal(c, ref["c_i"][iters - 1])
        e.close()
