"""MI355X parity at the BASELINE.json sizes (C3, C4, C5) against the CPU oracle.

The HIP path runs through the C ABI exactly as a chain does: hdpm_init_chain (la:27-77:
update_phi and the latent pool of N m entries, generated on the device), then Neal-8 sweeps
(n8:10-160), update_phi (cf:511-591), compute_loglikelihood (cf:379-401) and, for C3 / C4,
split-merge moves (sm:542-598, t = r = 10).  The oracle is the optimised restatement
(oracle/src/fast.c, fast = 2: bit-identical to the per-term restatement, tested on the
CPU in tests/test_oracle.py) fed the same state, pool and random stream.  Labels, K,
centers, sigmas and the 625-word stream must be bit-identical after every step; the
log-likelihood within rtol 1e-10 (north_star).

The split-merge moves at C3 / C4 overflow the reference's 2F1 series (hg:11-48: it throws
HDPM_E_GSL for clusters of ~1.4k+ members), so both sides run with the log-space extension
HDPM_OPT_HIG_LOGSPACE; that part is parity with the oracle's mirror of the
extension, not with the reference.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-10


@pytest.fixture(scope="module")
def hd():
    import split_and_merge_gibbs_sampling_amd as hd
    hd.build()
    return hd


def start(hd, oracle, name, seed, hig_log=False, phi_device=False):
    from split_and_merge_gibbs_sampling_amd.data import config
    ds = config(name)
    eng = hd.Engine(0)
    eng.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    eng.set_seed(seed)
    if hig_log:
        eng.set_hig_logspace(True)
    if phi_device:
        eng.set_phi_device(True)
    m = 3
    params = eng.chain_params(m=m, iterations=1, L=0, burnin=0, neal8=True, split_merge=hig_log, t=10, r=10)
    eng.init_chain(params, c_i=ds.truth)
    c, cen, sig = eng.get_state()
    P = ds.n * m
    pc, ps = eng.get_pool(P)
    ost = oracle.OracleState(c, cen.shape[0], cen, sig, cap=4096)
    return ds, eng, ost, eng.rng_state.copy(), pc, ps


def same(eng, ost, rng, what):
    c, cen, sig = eng.get_state()
    assert cen.shape[0] == ost.K, what
    assert np.array_equal(c, ost.c_i), what
    assert np.array_equal(cen, ost.centers[:ost.K]), what
    assert np.array_equal(sig, ost.sigma[:ost.K]), what
    assert np.array_equal(eng.rng_state, rng), what


def neal8_steps(eng, oracle, ds, ost, rng, pc, ps, sweeps):
    for k in range(sweeps):
        eng.neal8_sweep(3)
        assert oracle.neal8_sweep(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, ost, 3, pc, ps, rng, fast=2) == 0
        same(eng, ost, rng, f"sweep {k}")
        eng.update_phi()
        assert oracle.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, ost, rng) == 0
        same(eng, ost, rng, f"update_phi {k}")
        ll = eng.compute_loglikelihood()
        ref = oracle.compute_loglikelihood(ds.codes, ds.attrisize, ost, fast=2)
        np.testing.assert_allclose(ll, ref, rtol=RTOL, atol=0)


def sm_steps(eng, oracle, ds, ost, rng, moves, idx0=0):
    acc_total = 0
    for k in range(moves):
        acc = eng.split_and_merge(10, 10, idx0 + k)
        st, oacc = oracle.split_and_merge(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, ost, 10, 10, idx0 + k, rng,
                                          fast=2)
        assert st == 0
        assert acc == oacc, f"move {k}"
        same(eng, ost, rng, f"move {k}")
        acc_total += acc
    return acc_total


@pytest.mark.timeout(900)
def test_c5_full_size_sweeps(hd, oracle):
    """C5: N = 1,000,000, D = 128, m_j = 4, K = 20 (the bench workload)."""
    ds, eng, ost, rng, pc, ps = start(hd, oracle, "c5", seed=1)
    assert ds.n == 1_000_000 and ds.d == 128
    neal8_steps(eng, oracle, ds, ost, rng, pc, ps, sweeps=2)
    eng.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("phi_device", [False, True])
def test_c3_full_size_neal8_and_split_merge(hd, oracle, phi_device):
    """C3: N = 100,000, D = 64, m_j ~ U{2..6}, K = 20: Neal-8 + split-merge; with phi_device,
    update_phi on the device (BASELINE config C3: "hyperg phi-update on device")."""
    oracle.set_hig_logspace(True)
    if phi_device:
        os.environ["HDPM_PHI_TRACE"] = "1"        # a split-merge update handed back prints why
    try:
        ds, eng, ost, rng, pc, ps = start(hd, oracle, "c3", seed=2, hig_log=True, phi_device=phi_device)
        assert ds.n == 100_000 and ds.d == 64
        eng.reset_stats()
        neal8_steps(eng, oracle, ds, ost, rng, pc, ps, sweeps=2)
        if phi_device:
            st = eng.stats()
            assert st["phi_device_calls"] == 2 and st["phi_device_fallbacks"] == 0, st
        sm_steps(eng, oracle, ds, ost, rng, moves=4)
        if phi_device:
            # split-merge's update_phi({c1, c2}) (sm:221, 387, 584) on the device too
            st = eng.stats()
            # the split-merge updates run on the device; the ones handed back are drifts past
            # the widest window (a freshly split or merged cluster whose rhig draws reject ~90%
            # of their attempts: status 4 / 5), which the host job draws
            assert st["phi_sm_device_calls"] > 0 and (st["phi_fallback_status_mask"] & ~0x30) == 0, \
                {k: st[k] for k in ("phi_device_calls", "phi_device_fallbacks", "phi_sm_device_calls",
                                    "phi_device_last_status", "phi_fallback_status_mask", "phi_tree_calls",
                                    "phi_tree_retries", "sm_moves")}
        eng.close()
    finally:
        oracle.set_hig_logspace(False)


@pytest.mark.timeout(900)
def test_c4_full_size_neal8_and_split_merge(hd, oracle):
    """C4: MNIST surrogate N = 70,000, D = 784, m_j = 6 (wide rows: the generic prepass and
    the split-merge kernels at D = 784)."""
    oracle.set_hig_logspace(True)
    try:
        ds, eng, ost, rng, pc, ps = start(hd, oracle, "c4", seed=3, hig_log=True)
        assert ds.n == 70_000 and ds.d == 784
        neal8_steps(eng, oracle, ds, ost, rng, pc, ps, sweeps=2)
        eng.reset_stats()
        sm_steps(eng, oracle, ds, ost, rng, moves=3)
        # the restricted scans walked on many CUs (k_sm_scan_wide), none handed back
        st = eng.stats()
        if os.environ.get("HDPM_SM_WIDE") != "0":
            assert st["sm_wide_scans"] > 0 and st["sm_wide_fallbacks"] == 0, st
        eng.close()
    finally:
        oracle.set_hig_logspace(False)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("L", [1, 20])
# 0: the fixed-point resolver (k_resolve_fp); 4096: the one-wave LIST resolver without block
# mode; 8388608 (bit 23): the one-wave resolvers with block mode after many exact decisions;
# 1073741824 (bit 30): the device-wide fixed-point resolver (k_resolve_fpg) for every launch
@pytest.mark.parametrize("debug", [0, 4096, 8388608, 1073741824])
def test_c2_full_size_unconverged_starts(hd, oracle, L, debug):
    """C2: N = 10,000, D = 32, binary, from one cluster (L = 1) or a random assignment to 20
    labels (la:31-43, the scripts' L = 20): far from the posterior, points move every sweep
    and clusters appear and vanish (cases 2-4, resolver restarts)."""
    from split_and_merge_gibbs_sampling_amd.data import config
    ds = config("c2")
    eng = hd.Engine(0)
    eng.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    eng.set_seed(4)
    eng.set_debug(debug)
    params = eng.chain_params(m=3, iterations=1, L=L, burnin=0, neal8=True, split_merge=False)
    eng.init_chain(params, c_i=np.zeros(ds.n, np.int32) if L == 1 else None)
    c, cen, sig = eng.get_state()
    assert cen.shape[0] == L
    pc, ps = eng.get_pool(ds.n * 3)
    ost = oracle.OracleState(c, cen.shape[0], cen, sig, cap=8192)
    rng = eng.rng_state.copy()
    neal8_steps(eng, oracle, ds, ost, rng, pc, ps, sweeps=4)
    if L == 20:
        assert eng.stats()["moves"] > 0
    eng.close()


@pytest.mark.timeout(900)
# lat: the margin under which a latent kept as a head bound by the level-table exact rows counts
# as probability 0 (kernels.hip latent_fix); 1e9 sends every such latent to its exact sum
@pytest.mark.parametrize("lat", [None, 1e9])
def test_c5_full_size_random20_start(hd, oracle, lat):
    """C5 from a random assignment to 20 labels (la:31, the scripts' L = 20): every point is
    uncertain in the first sweeps; dense launches list every point, the level-table exact rows
    keep far-below latents as head bounds, the device-wide resolver decides them."""
    from split_and_merge_gibbs_sampling_amd.data import config
    ds = config("c5")
    eng = hd.Engine(0)
    eng.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    eng.set_seed(6)
    if lat:
        eng.set_lat_negligible(lat)
    params = eng.chain_params(m=3, iterations=1, L=20, burnin=0, neal8=True, split_merge=False)
    eng.init_chain(params, c_i=None)
    c, cen, sig = eng.get_state()
    pc, ps = eng.get_pool(ds.n * 3)
    ost = oracle.OracleState(c, cen.shape[0], cen, sig, cap=4096)
    rng = eng.rng_state.copy()
    neal8_steps(eng, oracle, ds, ost, rng, pc, ps, sweeps=2)
    st = eng.stats()
    assert st["moves"] > 100_000
    assert st["fpg_launches"] > 0, st     # the device-wide fixed-point resolver decided the sweeps
    assert st["dense_launches"] > 0, st
    eng.close()


@pytest.mark.timeout(1200)
# mode "": the default path; "nopipe": debug bit 22 (no sweep enqueued ahead of the update's
# go -- the same chain without the device-gated pipeline); "gateoff": the enqueued sweep's wait
# kernel gives up after 1 us with no host-side check, so nearly every enqueued sweep is gated
# off on the device and re-run ungated by the engine (its recovery path)
# "phidev": update_phi on the device (HDPM_OPT_PHI_DEVICE), speculated beside each sweep and
# committed when the sweep moved no point (engine.cpp dspec_launch / dspec_commit); "phigen": the
# same with the device's general kernels only (launch_phi, not the fast path launch_phi2);
# "host": the host job (the default -- automatic -- places C4's update on the device, C5's and
# C3's on the host)
@pytest.mark.parametrize("name,warm,timed,mode", [("c5", 5, 25, ""), ("c5", 3, 12, "nopipe"),
                                                  ("c5", 3, 12, "gateoff"), ("c5", 5, 25, "phidev"),
                                                  ("c3", 5, 25, ""), ("c3", 5, 25, "phidev"),
                                                  ("c4", 3, 25, ""), ("c4", 3, 15, "host"),
                                                  ("c4", 3, 10, "phigen")])
def test_bench_path_iterations_api(hd, oracle, name, warm, timed, mode):
    """The path bench.py times (bench.py main: hdpm_iterations for the warmup, synchronize,
    reset_stats, hdpm_iterations for the timed window) at the full BASELINE size, against
    the oracle's chain (la:94-132: sweep, update_phi, compute_loglikelihood per iteration,
    fast = 2).  Between two batches the next sweep stays prepared on the device (its prepass
    started at the end of the first batch, kRoundPrefix), and every iteration but the last of
    a batch launches the next sweep before its host work is done -- the pipelined code is
    what is compared here, not the one-call-per-step API.  The chain starts at iteration 1
    (iteration 0 regenerates the latent pool, la:123; the device pool generator has its own
    bit-exact tests), so the oracle reads the engine's pool once.  Per-iteration
    log-likelihoods, then labels, K, centers, sigmas and the 625-word stream after the timed
    batch, and again after a short batch that follows a get_state (which drops the prepared
    sweep) -- as launcher.cpp:85-132 would leave them."""
    ds, eng, ost, rng, pc, ps = start(hd, oracle, name, seed=11)
    if mode == "nopipe":
        eng.set_debug(4194304)
    elif mode == "gateoff":
        eng.set_pipe_wait_us(-1.0)
    elif mode == "phidev":
        eng.set_phi_device(True)
    elif mode == "phigen":
        eng.set_phi_device(True, general=True)
    elif mode == "host":
        eng.set_phi_device(False)
    params = eng.chain_params(m=3, iterations=warm + timed + 3, L=0, burnin=0, neal8=True, split_merge=False)
    eng._params = params

    def oracle_iters(it0, count):
        out = []
        for _ in range(count):
            assert oracle.neal8_sweep(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, ost, 3, pc, ps, rng, fast=2) == 0
            assert oracle.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, ost, rng) == 0
            out.append(oracle.compute_loglikelihood(ds.codes, ds.attrisize, ost, fast=2))
        return np.array(out)

    it = 1
    _, ll = eng.iterations(it, warm)
    it += warm
    if mode == "nopipe":
        eng.drop_prepared()                    # bench.py's window start (hdpm_drop_prepared)
    eng.synchronize()
    eng.reset_stats()
    np.testing.assert_allclose(ll, oracle_iters(it - warm, warm), rtol=RTOL, atol=0)
    _, ll = eng.iterations(it, timed)
    it += timed
    eng.synchronize()
    st = eng.stats()
    assert st["sweeps"] == timed
    if name == "c5" and mode == "":
        assert st["pipe_runs"] > 0, st          # the device-gated pipeline ran (engine.cpp pipe_go)
    if mode == "nopipe":
        assert st["pipe_enqueued"] == 0 and st["pipe_runs"] == 0, st
    if mode == "gateoff":
        assert st["pipe_recovered"] > 0, st
    dev = mode in ("phidev", "phigen") or (mode == "" and name == "c4")
    if dev:
        # every update on the device (none handed back to the host), from the speculation
        assert st["phi_device_calls"] == timed and st["phi_device_fallbacks"] == 0, st
        assert st["phi_dspec_used"] > 0, st
        if mode == "phigen":
            assert st["phi_fast_calls"] == 0, st
        else:
            assert st["phi_fast_calls"] >= timed and st["phi_fast_handbacks"] == 0, st
    else:
        assert st["phi_device_calls"] == 0, st
    np.testing.assert_allclose(ll, oracle_iters(it - timed, timed), rtol=RTOL, atol=0)
    same(eng, ost, rng, "after the timed batch")
    _, ll = eng.iterations(it, 3)
    np.testing.assert_allclose(ll, oracle_iters(it, 3), rtol=RTOL, atol=0)
    same(eng, ost, rng, "after a batch that follows get_state")
    eng.close()


@pytest.mark.timeout(900)
# fail_at k: workgroup 0 of every device-wide resolver launch gives up at its k-th grid barrier
# (k = 1, 2: the first round; later ordinals land in the later rounds, the drift / re-test
# barriers, the one before a window's commit and the one behind a stop); wait_us: a 1 us barrier
# limit, so that any barrier of any launch may give up
@pytest.mark.parametrize("fail_at,wait_us", [(1, 0.0), (2, 0.0), (3, 0.0), (4, 0.0), (5, 0.0), (6, 0.0), (7, 0.0),
                                             (9, 0.0), (12, 0.0), (17, 0.0), (0, 1.0)])
def test_c2_device_wide_resolver_gives_up_and_recovers(hd, oracle, fail_at, wait_us):
    """k_resolve_fpg's grid barriers are all-or-nothing (resolve_fpg.inl fpg::sync): a launch
    that gives up has committed exactly the windows before that barrier, reports a restart at
    its first undecided point, and the engine continues there on one workgroup (k_resolve_fp).
    Forced at every barrier ordinal of a launch, and by a 1 us limit, the chain (C2 from a
    random L = 20 start, the device-wide resolver for every fixed-point launch) stays
    bit-identical to the oracle (n8:10-160)."""
    from split_and_merge_gibbs_sampling_amd.data import config
    ds = config("c2")
    eng = hd.Engine(0)
    eng.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    eng.set_seed(4)
    eng.set_debug(1073741824)
    if fail_at:
        eng.set_fpg_fail_at(fail_at)
    if wait_us:
        eng.set_fpg_wait_us(wait_us)
    params = eng.chain_params(m=3, iterations=1, L=20, burnin=0, neal8=True, split_merge=False)
    eng.init_chain(params, c_i=None)
    c, cen, sig = eng.get_state()
    pc, ps = eng.get_pool(ds.n * 3)
    ost = oracle.OracleState(c, cen.shape[0], cen, sig, cap=8192)
    rng = eng.rng_state.copy()
    eng.reset_stats()
    neal8_steps(eng, oracle, ds, ost, rng, pc, ps, sweeps=3)
    st = eng.stats()
    assert st["fpg_launches"] > 0, st
    if fail_at:
        assert st["fpg_aborts"] > 0, st
    eng.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("kernel", [1, 2, 3])
def test_c2_unconverged_many_latents(hd, oracle, kernel):
    """m = 20 latent entries (E = K + m = 40 <= 64), C2 from a random L = 20 start, with
    snapshot draws, against the oracle, on each mass exact-rows kernel: the wave-per-point one
    (k_exact_rows_mass) takes a point's m + 1 > 16 draws from the stream per lane (ADVICE r4:
    its 16-word batch load picked the next point's words for latent u >= 16); the
    thread-per-point ones (compare / select, level tables) with k_snap_draws behind them."""
    from split_and_merge_gibbs_sampling_amd.data import config
    ds = config("c2")
    eng = hd.Engine(0)
    eng.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    eng.set_seed(8)
    m = 20
    eng.set_exact_kernel(kernel)
    params = eng.chain_params(m=m, iterations=1, L=20, burnin=0, neal8=True, split_merge=False)
    eng.init_chain(params, c_i=None)
    c, cen, sig = eng.get_state()
    pc, ps = eng.get_pool(ds.n * m)
    ost = oracle.OracleState(c, cen.shape[0], cen, sig, cap=8192)
    rng = eng.rng_state.copy()
    eng.reset_stats()
    for k in range(3):
        eng.neal8_sweep(m)
        assert oracle.neal8_sweep(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, ost, m, pc, ps, rng, fast=2) == 0
        same(eng, ost, rng, f"sweep {k}")
        eng.update_phi()
        assert oracle.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, ost, rng) == 0
        same(eng, ost, rng, f"update_phi {k}")
    st = eng.stats()
    assert st["exact_mass_launches" if kernel == 1 else "exact_lanes_launches"] > 0, st
    eng.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("lat", [40.0, 1e9])
def test_c2_latent_bounds(hd, oracle, lat):
    """C2 from a random L = 20 start with the level-table exact rows and latent head bounds:
    at the default margin (40) a bounded latent counts as probability 0, at 1e9 every bounded
    latent is summed exactly when a draw reads it (kernels.hip latent_fix / latent_exact, in the
    snapshot draws, both fixed-point resolvers and the serial path)."""
    from split_and_merge_gibbs_sampling_amd.data import config
    ds = config("c2")
    eng = hd.Engine(0)
    eng.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    eng.set_seed(12)
    eng.set_exact_kernel(3)
    eng.set_lat_negligible(lat)
    params = eng.chain_params(m=3, iterations=1, L=20, burnin=0, neal8=True, split_merge=False)
    eng.init_chain(params, c_i=None)
    c, cen, sig = eng.get_state()
    pc, ps = eng.get_pool(ds.n * 3)
    ost = oracle.OracleState(c, cen.shape[0], cen, sig, cap=8192)
    rng = eng.rng_state.copy()
    eng.reset_stats()
    neal8_steps(eng, oracle, ds, ost, rng, pc, ps, sweeps=4)
    assert eng.stats()["exact_lanes_launches"] > 0
    eng.close()
