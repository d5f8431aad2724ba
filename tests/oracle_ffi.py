"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product (split_and_merge_gibbs_sampling_amd) never imports this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


class ChainParams(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "verbose", "m", "iterations", "L", "burnin", "t", "r", "neal8", "split_merge",
        "n8_step_size", "sam_step_size", "thinning", "fast")]


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        L.orc_ffi_set_seed.argtypes = [C.c_uint32, _i32p]
        L.orc_ffi_set_hig_logspace.argtypes = [C.c_int]
        L.orc_ffi_set_hig_logspace.restype = None
        L.orc_ffi_runif.argtypes = [_i32p, C.c_int64, _f64p]
        L.orc_ffi_rbeta.argtypes = [_i32p, C.c_double, C.c_double, C.c_int, _f64p]
        L.orc_ffi_rhig.argtypes = [_i32p, C.c_double, C.c_double, C.c_double, C.c_int, _f64p]
        L.orc_ffi_sample_prob1.argtypes = [_i32p, _f64p, C.c_int, C.POINTER(C.c_int)]
        L.orc_ffi_norm_const2.argtypes = [C.c_double, C.c_double, C.c_double, C.POINTER(C.c_int)]
        L.orc_ffi_norm_const2.restype = C.c_double
        L.orc_ffi_qbeta01_lt.argtypes = [C.c_double, C.c_double, C.c_double]
        L.orc_ffi_pbeta.argtypes = [C.c_double, C.c_double, C.c_double]
        L.orc_ffi_pbeta.restype = C.c_double
        L.orc_ffi_dhamming.argtypes = [C.c_int, C.c_int, C.c_double, C.c_int]
        L.orc_ffi_dhamming.restype = C.c_double
        L.orc_ffi_loglik_matrix.argtypes = [_f64p, C.c_int, C.c_int, _i32p, _f64p, _f64p, C.c_int,
                                            _f64p, _i32p]
        L.orc_ffi_neal8_sweep.argtypes = [_f64p, C.c_int, C.c_int, _i32p, C.c_double, _f64p, _f64p,
                                          _i32p, C.POINTER(C.c_int), _f64p, _f64p, C.c_int, C.c_int,
                                          _f64p, _f64p, C.c_int64, _i32p, C.c_int, C.c_int, C.c_int]
        L.orc_ffi_update_phi.argtypes = [_f64p, C.c_int, C.c_int, _i32p, _f64p, _f64p, _i32p, C.c_int,
                                         _f64p, _f64p, C.c_void_p, C.c_int, _i32p]
        L.orc_ffi_compute_loglikelihood.argtypes = [_f64p, C.c_int, C.c_int, _i32p, _i32p, C.c_int,
                                                    _f64p, _f64p]
        L.orc_ffi_compute_loglikelihood.restype = C.c_double
        L.orc_ffi_compute_loglikelihood_opt.argtypes = L.orc_ffi_compute_loglikelihood.argtypes
        L.orc_ffi_compute_loglikelihood_opt.restype = C.c_double
        L.orc_ffi_set_threads.argtypes = [C.c_int]
        L.orc_ffi_set_threads.restype = None
        L.orc_ffi_pool_generate.argtypes = [_i32p, C.c_int, _f64p, _f64p, C.c_int64, _f64p, _f64p,
                                            _i32p]
        L.orc_ffi_restricted_gibbs.argtypes = [_f64p, C.c_int, C.c_int, _i32p, _f64p, _f64p, _i32p,
                                               C.c_int, _i32p, C.c_int, _f64p, _f64p, C.c_int, C.c_int,
                                               C.c_int, _i32p, C.c_int]
        L.orc_ffi_logprobgs_c_i.argtypes = [_f64p, C.c_int, C.c_int, _i32p, _i32p, _f64p, _f64p,
                                            C.c_int, _i32p, _i32p, C.c_int, C.c_int, C.c_int]
        L.orc_ffi_logprobgs_c_i.restype = C.c_double
        L.orc_ffi_split_and_merge.argtypes = [_f64p, C.c_int, C.c_int, _i32p, C.c_double, _f64p, _f64p,
                                              _i32p, C.POINTER(C.c_int), _f64p, _f64p, C.c_int, C.c_int,
                                              C.c_int, C.c_int, _i32p, C.c_int, C.POINTER(C.c_int)]
        L.orc_run_markov_chain.argtypes = [_f64p, C.c_int, C.c_int, _i32p, C.c_double, _f64p, _f64p,
                                           C.POINTER(ChainParams), C.c_void_p, _i32p, _i32p, _i32p,
                                           _f64p, _i32p, _i32p]
        _lib = L
    return _lib


# ----------------------------------------------------------------- RNG
def seed_state(seed: int) -> np.ndarray:
    st = np.zeros(625, np.int32)
    lib().orc_ffi_set_seed(seed & 0xFFFFFFFF, st)
    return st


def runif(state: np.ndarray, n: int) -> np.ndarray:
    out = np.zeros(n, np.float64)
    lib().orc_ffi_runif(state, n, out)
    return out


def rbeta(state, a, b, n):
    out = np.zeros(n, np.float64)
    lib().orc_ffi_rbeta(state, a, b, n, out)
    return out


def rhig(state, v, w, m, n):
    out = np.zeros(n, np.float64)
    st = lib().orc_ffi_rhig(state, v, w, m, n, out)
    return out, st


def sample_prob1(state, probs):
    idx = C.c_int(-1)
    p = np.ascontiguousarray(probs, np.float64)
    st = lib().orc_ffi_sample_prob1(state, p, len(p), C.byref(idx))
    return idx.value, st


def norm_const2(d, c, m):
    err = C.c_int(0)
    v = lib().orc_ffi_norm_const2(d, c, m, C.byref(err))
    return v, err.value


def set_hig_logspace(on: bool):
    """Mirror of hdpm's HDPM_OPT_HIG_LOGSPACE extension (process-wide in the oracle)."""
    lib().orc_ffi_set_hig_logspace(1 if on else 0)


# ----------------------------------------------------------------- model
_cm_cache = {}


def colmajor(codes: np.ndarray) -> np.ndarray:
    """N x D integer codes -> column-major float64 buffer (Rcpp::NumericMatrix layout).
    The last large conversion is memoised (the BASELINE-size cases reuse one matrix)."""
    codes = np.asarray(codes)
    if codes.size < 1_000_000:
        return np.ascontiguousarray(np.asarray(codes, np.float64).T).reshape(-1)
    key = (codes.__array_interface__["data"][0], codes.shape, codes.strides, codes.dtype.str)
    hit = _cm_cache.get(key)
    if hit is None or hit[0] is not codes:
        _cm_cache.clear()
        hit = (codes, np.ascontiguousarray(np.asarray(codes, np.float64).T).reshape(-1))
        _cm_cache[key] = hit
    return hit[1]


def set_threads(n: int):
    """OpenMP threads of the optimised oracle (fast=2); 0 = the runtime default."""
    lib().orc_ffi_set_threads(int(n))


def loglik_matrix(codes, attrisize, centers, sigma):
    codes = np.asarray(codes)
    n, d = codes.shape
    K = centers.shape[0]
    L = np.zeros((n, K), np.float64)
    H = np.zeros((n, K), np.int32)
    lib().orc_ffi_loglik_matrix(colmajor(codes), n, d, np.ascontiguousarray(attrisize, np.int32),
                                np.ascontiguousarray(centers, np.float64),
                                np.ascontiguousarray(sigma, np.float64), K, L.reshape(-1), H.reshape(-1))
    return L, H


class OracleState:
    """Mutable chain state (c_i, K, centers[cap x d], sigma[cap x d]) for ffi calls."""

    def __init__(self, c_i, K, centers, sigma, cap=None):
        n = len(c_i)
        d = centers.shape[1]
        cap = cap or (n + 2)          # BASELINE-size cases pass a smaller cap (clusters, not points)
        self.c_i = np.ascontiguousarray(c_i, np.int32).copy()
        self.K = int(K)
        self.centers = np.zeros((cap, d), np.float64)
        self.sigma = np.zeros((cap, d), np.float64)
        self.centers[:K] = centers[:K]
        self.sigma[:K] = sigma[:K]
        self.cap = cap

    def copy(self):
        return OracleState(self.c_i, self.K, self.centers, self.sigma, self.cap)


def neal8_sweep(codes, attrisize, gamma, v, w, state: OracleState, m, pool_center, pool_sigma,
                rng, fast=1, first=0, count=-1):
    codes = np.asarray(codes)
    n, d = codes.shape
    K = C.c_int(state.K)
    st = lib().orc_ffi_neal8_sweep(colmajor(codes), n, d, np.ascontiguousarray(attrisize, np.int32),
                                   gamma, np.ascontiguousarray(v, np.float64),
                                   np.ascontiguousarray(w, np.float64), state.c_i, C.byref(K),
                                   state.centers.reshape(-1), state.sigma.reshape(-1), state.cap, m,
                                   np.ascontiguousarray(pool_center, np.float64).reshape(-1),
                                   np.ascontiguousarray(pool_sigma, np.float64).reshape(-1),
                                   pool_center.shape[0], rng, fast, first, count)
    state.K = K.value
    return st


def update_phi(codes, attrisize, v, w, state: OracleState, rng, idx=None):
    codes = np.asarray(codes)
    n, d = codes.shape
    K = state.K
    cen = np.ascontiguousarray(state.centers[:K])
    sig = np.ascontiguousarray(state.sigma[:K])
    if idx is None:
        ip, ni = None, 0
    else:
        ia = np.ascontiguousarray(idx, np.int32)
        ip, ni = ia.ctypes.data, len(ia)
    st = lib().orc_ffi_update_phi(colmajor(codes), n, d, np.ascontiguousarray(attrisize, np.int32),
                                  np.ascontiguousarray(v, np.float64), np.ascontiguousarray(w, np.float64),
                                  state.c_i, K, cen.reshape(-1), sig.reshape(-1), ip, ni, rng)
    state.centers[:K] = cen
    state.sigma[:K] = sig
    return st


def compute_loglikelihood(codes, attrisize, state: OracleState, fast=1):
    codes = np.asarray(codes)
    n, d = codes.shape
    f = lib().orc_ffi_compute_loglikelihood_opt if fast >= 2 else lib().orc_ffi_compute_loglikelihood
    return f(colmajor(codes), n, d,
                                               np.ascontiguousarray(attrisize, np.int32), state.c_i,
                                               state.K, np.ascontiguousarray(state.centers[:state.K]).reshape(-1),
                                               np.ascontiguousarray(state.sigma[:state.K]).reshape(-1))


def pool_generate(attrisize, v, w, P, rng):
    d = len(attrisize)
    pc = np.zeros((P, d), np.float64)
    ps = np.zeros((P, d), np.float64)
    st = lib().orc_ffi_pool_generate(np.ascontiguousarray(attrisize, np.int32), d,
                                     np.ascontiguousarray(v, np.float64), np.ascontiguousarray(w, np.float64),
                                     P, pc.reshape(-1), ps.reshape(-1), rng)
    return pc, ps, st


def restricted_gibbs(codes, attrisize, v, w, S, state: OracleState, i1, i2, t, rng, fast=1):
    codes = np.asarray(codes)
    n, d = codes.shape
    K = state.K
    cen = np.ascontiguousarray(state.centers[:K])
    sig = np.ascontiguousarray(state.sigma[:K])
    Sa = np.ascontiguousarray(S, np.int32)
    st = lib().orc_ffi_restricted_gibbs(colmajor(codes), n, d, np.ascontiguousarray(attrisize, np.int32),
                                        np.ascontiguousarray(v, np.float64), np.ascontiguousarray(w, np.float64),
                                        Sa, len(Sa), state.c_i, K, cen.reshape(-1), sig.reshape(-1),
                                        i1, i2, t, rng, fast)
    state.centers[:K] = cen
    state.sigma[:K] = sig
    return st


def logprobgs_c_i(codes, attrisize, gs: OracleState, g_c_i, S, i1, i2):
    codes = np.asarray(codes)
    n, d = codes.shape
    Sa = np.ascontiguousarray(S, np.int32)
    return lib().orc_ffi_logprobgs_c_i(colmajor(codes), n, d, np.ascontiguousarray(attrisize, np.int32),
                                       gs.c_i, np.ascontiguousarray(gs.centers[:gs.K]).reshape(-1),
                                       np.ascontiguousarray(gs.sigma[:gs.K]).reshape(-1), gs.K,
                                       np.ascontiguousarray(g_c_i, np.int32), Sa, len(Sa), i1, i2)


def split_and_merge(codes, attrisize, gamma, v, w, state: OracleState, t, r, idx_1_sm, rng, fast=1):
    codes = np.asarray(codes)
    n, d = codes.shape
    K = C.c_int(state.K)
    acc = C.c_int(0)
    st = lib().orc_ffi_split_and_merge(colmajor(codes), n, d, np.ascontiguousarray(attrisize, np.int32),
                                       gamma, np.ascontiguousarray(v, np.float64),
                                       np.ascontiguousarray(w, np.float64), state.c_i, C.byref(K),
                                       state.centers.reshape(-1), state.sigma.reshape(-1), state.cap,
                                       t, r, idx_1_sm, rng, fast, C.byref(acc))
    state.K = K.value
    return st, acc.value


def run_markov_chain(codes, attrisize, gamma, v, w, *, m=5, iterations=1000, L=1, c_i=None,
                     burnin=5000, t=10, r=10, neal8=False, split_merge=True, n8_step_size=1,
                     sam_step_size=1, thinning=1, rng=None, seed=None, fast=1):
    """Oracle restatement of run_markov_chain (la:6-174).  Returns (status, results dict)."""
    codes = np.asarray(codes)
    n, d = codes.shape
    if rng is None:
        rng = seed_state(seed if seed is not None else 0)
    p = ChainParams(0, m, iterations, L, burnin, t, r, int(neal8), int(split_merge), n8_step_size,
                    sam_step_size, thinning, int(fast))
    tot = np.zeros(iterations, np.int32)
    cis = np.zeros((iterations, n), np.int32)
    ll = np.zeros(iterations, np.float64)
    acc = np.zeros(iterations, np.int32)
    fin = np.zeros(n, np.int32)
    if c_i is not None:
        ci = np.ascontiguousarray(c_i, np.int32)
        cptr = ci.ctypes.data
    else:
        ci, cptr = None, None
    st = lib().orc_run_markov_chain(colmajor(codes), n, d, np.ascontiguousarray(attrisize, np.int32),
                                    gamma, np.ascontiguousarray(v, np.float64),
                                    np.ascontiguousarray(w, np.float64), C.byref(p), cptr, rng, tot,
                                    cis.reshape(-1), ll, acc, fin)
    return st, {"total_cls": tot, "c_i": cis, "loglikelihood": ll, "accepted": acc, "final_ass": fin}
