"""Host-side mirror of the reference sampler's interface on the MI355X engine.

``run_markov_chain`` keeps the signature and result fields of the reference's Rcpp
export (code/launcher.cpp:6-14, 57-63, 170-173); ``Engine`` exposes the C++ entry points
of the hot path (sample_allocation sweep, update_phi, compute_loglikelihood,
split_restricted_gibbs_sampler, logprobgs_c_i, split_and_merge) over the C ABI.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import HdpmError, ptr


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class Engine:
    """One hdpm context (one GPU, one chain, one R random stream)."""

    def __init__(self, device: int = 0):
        L = _lib.lib()
        h = C.c_void_p()
        st = L.hdpm_ctx_create(device, C.byref(h))
        if st != 0:
            raise HdpmError(st, f"cannot create a context on device {device} (needs a gfx950 GPU)")
        self._L, self._h = L, h
        self.n = self.d = 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.hdpm_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st):
        if st != 0:
            raise HdpmError(st, self._L.hdpm_last_error(self._h).decode())

    # ---------------------------------------------------------------- data / rng / state
    def set_data(self, codes, attrisize, gamma, v, w):
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        self.n, self.d = codes.shape
        self._att = _i32(attrisize)
        self._keep = (codes, self._att, _f64(v), _f64(w))
        self._check(self._L.hdpm_set_data(self._h, ptr(codes), self.n, self.d, ptr(self._att), float(gamma),
                                          ptr(self._keep[2]), ptr(self._keep[3])))

    def set_seed(self, seed: int):
        self._check(self._L.hdpm_rng_set_seed(self._h, seed & 0xFFFFFFFF))

    @property
    def rng_state(self) -> np.ndarray:
        s = np.zeros(625, np.int32)
        self._check(self._L.hdpm_rng_get_state(self._h, ptr(s)))
        return s

    @rng_state.setter
    def rng_state(self, s):
        s = _i32(s)
        self._check(self._L.hdpm_rng_set_state(self._h, ptr(s)))

    def rng_fill_device(self, count: int) -> np.ndarray:
        """`count` raw MT outputs generated on the device (advances the stream)."""
        out = np.zeros(count, np.uint32)
        self._check(self._L.hdpm_rng_fill_device(self._h, int(count), ptr(out)))
        return out

    def set_state(self, c_i, centers, sigma):
        c = _i32(c_i)
        cen, sig = _f64(centers), _f64(sigma)
        self._check(self._L.hdpm_set_state(self._h, ptr(c), cen.shape[0], ptr(cen), ptr(sig)))

    def get_state(self):
        c = np.zeros(self.n, np.int32)
        K = C.c_int32(0)
        self._check(self._L.hdpm_get_state(self._h, ptr(c), C.byref(K), None, None, 0))
        cen = np.zeros((K.value, self.d))
        sig = np.zeros((K.value, self.d))
        self._check(self._L.hdpm_get_state(self._h, ptr(c), C.byref(K), ptr(cen), ptr(sig), K.value))
        return c, cen, sig

    def set_pool(self, centers, sigma):
        cen, sig = _f64(centers), _f64(sigma)
        self._check(self._L.hdpm_set_pool(self._h, ptr(cen), ptr(sig), cen.shape[0]))

    def generate_pool(self, P: int):
        self._check(self._L.hdpm_generate_pool(self._h, int(P)))

    def get_pool(self, P: int):
        cen = np.zeros((P, self.d))
        sig = np.zeros((P, self.d))
        self._check(self._L.hdpm_get_pool(self._h, ptr(cen), ptr(sig), int(P)))
        return cen, sig

    def get_pool_heads(self, P: int) -> np.ndarray:
        """The prepass's pool-entry heads, P x stride uint64 words, wb Ws + 2 of them used
        (diagnostics; csrc/kernels.hpp "Pool-entry heads")."""
        mmax = int(self._att.max())
        wb = 1 if mmax <= 2 else 2 if mmax <= 4 else 4 if mmax <= 16 else 8
        wd = -(-self.d // 64)
        Ws = 2 if wd <= 2 else 4 if wd <= 4 else wd
        hw = wb * Ws + 2
        if Ws == 2 or (Ws == 4 and wb <= 4):      # kernels.hpp head_stride
            stride = 4
            while stride < hw:
                stride *= 2
        else:
            stride = -(-hw // 8) * 8
        out = np.zeros((P, stride), np.uint64)
        self._check(self._L.hdpm_get_pool_heads(self._h, ptr(out), int(P)))
        return out

    # ---------------------------------------------------------------- hot path
    def neal8_sweep(self, m: int):
        """N sample_allocation calls in index order (code/launcher.cpp:95-99)."""
        self._check(self._L.hdpm_neal8_sweep(self._h, int(m)))

    def update_phi(self, cluster_indexes=None):
        if cluster_indexes is None:
            self._check(self._L.hdpm_update_phi(self._h, None, 0))
        else:
            idx = _i32(cluster_indexes)
            self._check(self._L.hdpm_update_phi(self._h, ptr(idx), len(idx)))

    def compute_loglikelihood(self) -> float:
        out = C.c_double(0.0)
        self._check(self._L.hdpm_compute_loglikelihood(self._h, C.byref(out)))
        return out.value

    def loglik_matrix(self, K: int):
        Lm = np.zeros((self.n, K))
        H = np.zeros((self.n, K), np.int32)
        self._check(self._L.hdpm_loglik_matrix(self._h, ptr(Lm), ptr(H)))
        return Lm, H

    def restricted_gibbs(self, S, i1, i2, t=1):
        S = _i32(S)
        self._check(self._L.hdpm_restricted_gibbs(self._h, ptr(S), len(S), int(i1), int(i2), int(t)))

    def logprobgs_c_i(self, g_c_i, S, i1, i2) -> float:
        g, S = _i32(g_c_i), _i32(S)
        out = C.c_double(0.0)
        self._check(self._L.hdpm_logprobgs_c_i(self._h, ptr(g), ptr(S), len(S), int(i1), int(i2), C.byref(out)))
        return out.value

    def split_and_merge(self, t, r, idx_1_sm=0) -> int:
        acc = C.c_int32(0)
        self._check(self._L.hdpm_split_and_merge(self._h, int(t), int(r), int(idx_1_sm), C.byref(acc)))
        return acc.value

    def stats(self) -> dict:
        s = _lib.Stats()
        self._check(self._L.hdpm_get_stats(self._h, C.byref(s)))
        return s.as_dict()

    def reset_stats(self):
        self._check(self._L.hdpm_reset_stats(self._h))

    def set_debug(self, mode: int):
        self._check(self._L.hdpm_set_debug(self._h, int(mode)))

    def synchronize(self):
        self._check(self._L.hdpm_synchronize(self._h))

    def drop_prepared(self):
        """Drop a prepared next sweep (include/hdpm.h hdpm_drop_prepared): the next iteration
        does all of its own work."""
        self._check(self._L.hdpm_drop_prepared(self._h))

    def debug_draw(self, logw, rU: float, two_way: bool = False, ocml: bool = False) -> int:
        """Testing: one device draw from log-weights (n8:95-102, or the sm:204-215 two-way
        draw) with the engine's glibc exp, or the device libm's (ocml)."""
        w = _f64(logw)
        pick = C.c_int32(0)
        self._check(self._L.hdpm_debug_draw(self._h, _lib.ptr(w), int(w.size), float(rU), int(two_way), int(ocml),
                                            C.byref(pick)))
        return pick.value

    def debug_math(self, x, fn: str = "exp", ocml: bool = False) -> np.ndarray:
        """Testing: exp / log of x on the device (glibc's algorithm, or the device libm's)."""
        xs = _f64(x).ravel()
        out = np.empty_like(xs)
        self._check(self._L.hdpm_debug_math(self._h, _lib.ptr(xs), int(xs.size), 0 if fn == "exp" else 1,
                                            int(ocml), _lib.ptr(out)))
        return out

    def set_phi_device(self, on=True, general: bool = False):
        """update_phi on the device (include/hdpm.h HDPM_OPT_PHI_DEVICE); same chain.  on: True
        (device), False (host job), or "auto" (the default: device for updates of >= 4096 items);
        general: the device's general kernels only (launch_phi), not the fast path (launch_phi2)."""
        v = 3.0 if on == "auto" else (2.0 if general else 1.0) if on else 0.0
        self._check(self._L.hdpm_set_option(self._h, _lib.OPT_PHI_DEVICE, v))

    def get_option(self, option: int) -> float:
        """The current value of an include/hdpm.h HDPM_OPT_* option (hdpm_get_option)."""
        v = C.c_double()
        self._check(self._L.hdpm_get_option(self._h, int(option), C.byref(v)))
        return float(v.value)

    @property
    def phi_mode(self) -> str:
        """Where update_phi runs (HDPM_OPT_PHI_DEVICE): "host", "device", "device-general" or "auto"."""
        return {0: "host", 1: "device", 2: "device-general", 3: "auto"}[int(self.get_option(_lib.OPT_PHI_DEVICE))]

    def set_pipe_wait_us(self, us: float):
        """Testing (include/hdpm.h HDPM_OPT_PIPE_WAIT_US): the wait limit of a sweep enqueued
        ahead; negative: no host-side check (exercises the device gate-off recovery)."""
        self._check(self._L.hdpm_set_option(self._h, _lib.OPT_PIPE_WAIT_US, float(us)))

    def set_fpg_wait_us(self, us: float):
        """The grid-barrier limit of the device-wide resolver (include/hdpm.h
        HDPM_OPT_FPG_WAIT_US); a launch that gives up is continued on one workgroup."""
        self._check(self._L.hdpm_set_option(self._h, _lib.OPT_FPG_WAIT_US, float(us)))

    def set_fpg_fail_at(self, k: int):
        """Testing (include/hdpm.h HDPM_OPT_FPG_FAIL_AT): every device-wide resolver launch gives
        up at its k-th grid barrier (0: never)."""
        self._check(self._L.hdpm_set_option(self._h, _lib.OPT_FPG_FAIL_AT, float(k)))

    def set_exact_kernel(self, which: int):
        """Testing (include/hdpm.h HDPM_OPT_EXACT_KERNEL): 0 automatic, 1 a wave per point, 2 a
        thread per point, 3 level-indexed tables."""
        self._check(self._L.hdpm_set_option(self._h, _lib.OPT_EXACT_KERNEL, float(which)))

    def set_lat_negligible(self, margin: float):
        """Testing (include/hdpm.h HDPM_OPT_LAT_NEGLIGIBLE): the margin under which a latent
        kept as a head bound counts as probability 0 (>= 40; larger: exact sums instead)."""
        self._check(self._L.hdpm_set_option(self._h, _lib.OPT_LAT_NEGLIGIBLE, float(margin)))

    def set_sm_wide_wait_us(self, us: float):
        """Testing (include/hdpm.h HDPM_OPT_SM_WIDE_WAIT_US): the grid-barrier limit of the
        split-merge scan on many CUs; 0 gives up at once (the one-workgroup scan runs)."""
        self._check(self._L.hdpm_set_option(self._h, _lib.OPT_SM_WIDE_WAIT_US, float(us)))

    def set_sm_chain(self, mode: int):
        """include/hdpm.h HDPM_OPT_SM_CHAIN: the restricted Gibbs sampler as one device chain (1)
        or scan by scan (0, default); testing: 2 + 3k / 3 + 3k / 4 + 3k stop the chain at scan k / its
        lower / larger label's update."""
        self._check(self._L.hdpm_set_option(self._h, _lib.OPT_SM_CHAIN, float(mode)))

    def set_hig_logspace(self, on: bool = True):
        """Extension beyond the reference (include/hdpm.h HDPM_OPT_HIG_LOGSPACE): finite HIG
        log-densities for clusters whose 2F1 series overflows (the reference throws)."""
        self._check(self._L.hdpm_set_option(self._h, _lib.OPT_HIG_LOGSPACE, 1.0 if on else 0.0))

    # ---------------------------------------------------------------- driver
    @staticmethod
    def chain_params(verbose=0, m=5, iterations=1000, L=1, burnin=5000, t=10, r=10, neal8=False,
                     split_merge=True, n8_step_size=1, sam_step_size=1, thinning=1):
        return _lib.ChainParams(verbose, m, iterations, L, burnin, t, r, int(bool(neal8)), int(bool(split_merge)),
                                n8_step_size, sam_step_size, thinning)

    def init_chain(self, params, c_i=None):
        """code/launcher.cpp:27-77 (initial state, update_phi, latent pool)."""
        self._params = params
        self._idx_1_sm = C.c_int32(0)
        ci = None if c_i is None else _i32(c_i)
        self._check(self._L.hdpm_init_chain(self._h, C.byref(params), ptr(ci)))

    def iteration(self, it: int):
        """One pass of the loop body code/launcher.cpp:85-132; returns (accepted, loglik)."""
        acc = C.c_int32(0)
        ll = C.c_double(0.0)
        self._check(self._L.hdpm_iteration(self._h, C.byref(self._params), int(it), C.byref(self._idx_1_sm),
                                           C.byref(acc), C.byref(ll)))
        return acc.value, ll.value

    def iterations(self, it0: int, count: int):
        """Iterations it0 .. it0+count-1 in one call (the next sweep is launched while the
        host finishes the current iteration); returns (accepted[count], loglik[count])."""
        acc = np.zeros(count, np.int32)
        ll = np.zeros(count, np.float64)
        self._check(self._L.hdpm_iterations(self._h, C.byref(self._params), int(it0), int(count),
                                            C.byref(self._idx_1_sm), ptr(acc), ptr(ll)))
        return acc, ll

    def iterations_record(self, it0: int, count: int, labels: bool = True, out=None):
        """Iterations it0 .. it0+count-1 with the saved ones recorded (hdpm_iterations_record,
        la:139-153): (accepted[count], loglik[count], total_cls[saved], c_i[saved, n] or None,
        centers / sigmas: lists of K x D arrays per saved iteration).  out: a preallocated
        int32 (>= count) x n array for the labels (reused by bench.py --record)."""
        acc = np.zeros(count, np.int32)
        ll = np.zeros(count, np.float64)
        tot = np.zeros(count, np.int32)
        if out is not None:
            assert out.dtype == np.int32 and out.shape[0] >= count and out.shape[1] == self.n and out.flags.c_contiguous
            cis = out
        else:
            cis = np.zeros((count, self.n), np.int32) if labels else None
        ns = C.c_int32(0)
        self._check(self._L.hdpm_iterations_record(self._h, C.byref(self._params), int(it0), int(count),
                                                   C.byref(self._idx_1_sm), ptr(acc), ptr(ll), ptr(tot), ptr(cis),
                                                   C.byref(ns)))
        s = ns.value
        rows = C.c_int64(0)
        self._check(self._L.hdpm_record_take(self._h, None, None, C.byref(rows)))
        cen = np.zeros((rows.value, self.d), np.float64)
        sig = np.zeros((rows.value, self.d), np.float64)
        self._check(self._L.hdpm_record_take(self._h, ptr(cen), ptr(sig), C.byref(rows)))
        off = np.concatenate([[0], np.cumsum(tot[:s])])
        cens = [cen[off[q]:off[q + 1]] for q in range(s)]
        sigs = [sig[off[q]:off[q + 1]] for q in range(s)]
        return acc, ll, tot[:s], (cis[:s] if labels else None), cens, sigs

    def run_markov_chain(self, *, verbose=0, m=5, iterations=1000, L=1, c_i=None, burnin=5000, t=10, r=10,
                         neal8=False, split_merge=True, n8_step_size=1, sam_step_size=1, thinning=1,
                         keep_params=False):
        p = _lib.ChainParams(verbose, m, iterations, L, burnin, t, r, int(bool(neal8)), int(bool(split_merge)),
                             n8_step_size, sam_step_size, thinning)
        if keep_params:
            return self._run_recording(p, c_i)
        tot = np.zeros(iterations, np.int32)
        cis = np.zeros((iterations, self.n), np.int32)
        ll = np.zeros(iterations, np.float64)
        acc = np.zeros(iterations, np.int32)
        fin = np.zeros(self.n, np.int32)
        tm = np.zeros(1, np.float64)
        ci = None if c_i is None else _i32(c_i)
        self._check(self._L.hdpm_run_markov_chain(self._h, C.byref(p), ptr(ci), ptr(tot), ptr(cis), ptr(ll),
                                                  ptr(acc), ptr(fin), ptr(tm)))
        return {"total_cls": tot, "c_i": cis, "loglikelihood": ll, "final_ass": fin,
                "time": float(tm[0]), "accepted": acc}

    def _run_recording(self, p, c_i, chunk: int = 256):
        """The la:85-154 loop with the cluster parameters of every saved iteration recorded as
        the reference does (centers / sigmas, la:144-147: K x D arrays): hdpm_init_chain, then
        hdpm_iterations_record in batches (the pipelined sweeps keep running across saved
        iterations)."""
        import time
        iterations, burnin, thinning = p.iterations, p.burnin, p.thinning
        tot = np.zeros(iterations, np.int32)
        cis = np.zeros((iterations, self.n), np.int32)
        ll = np.zeros(iterations, np.float64)
        acc = np.zeros(iterations, np.int32)
        cens, sigs = [None] * iterations, [None] * iterations
        t0 = time.perf_counter()
        self.init_chain(p, c_i)
        total = (iterations + burnin) * thinning
        it = 0
        while it < total:
            cnt = min(chunk, total - it)
            a, lik, kk, cc, cen, sig = self.iterations_record(it, cnt)
            q = 0
            for k in range(cnt):
                i = it + k
                if i >= thinning * burnin and i % thinning == 0:
                    at = i // thinning - burnin
                    tot[at], cis[at], ll[at], acc[at] = kk[q], cc[q], lik[k], a[k]
                    cens[at], sigs[at] = cen[q], sig[q]
                    q += 1
            it += cnt
        fin = self.get_state()[0]
        return {"total_cls": tot, "c_i": cis, "centers": cens, "sigmas": sigs, "loglikelihood": ll,
                "final_ass": fin, "time": time.perf_counter() - t0, "accepted": acc}


def run_markov_chain(data, attrisize, gamma, v, w, verbose=0, m=5, iterations=1000, L=1, c_i=None,
                     burnin=5000, t=10, r=10, neal8=False, split_merge=True, n8_step_size=1,
                     sam_step_size=1, thinning=1, *, seed=None, rng_state=None, device=0, hig_logspace=False,
                     keep_params=False):
    """Drop-in for the reference's ``run_markov_chain`` (code/launcher.cpp:6-14).

    ``data`` holds the categorical codes 1..m_j (an N x D matrix).  The R random stream
    is ``set.seed(seed)`` or an explicit 625-word ``rng_state``; the returned dict has
    the fields of the reference's result list (plus ``rng_state`` after the run).
    ``hig_logspace=True`` turns on the log-space 2F1 extension (``Engine.set_hig_logspace``);
    the default keeps the reference's semantics, including its throw on overflow.
    ``keep_params=True`` also returns ``centers`` / ``sigmas`` of every saved iteration
    (la:144-147), running the loop iteration by iteration.
    """
    eng = Engine(device)
    try:
        eng.set_data(np.asarray(data), attrisize, gamma, v, w)
        if hig_logspace:
            eng.set_hig_logspace(True)
        if rng_state is not None:
            eng.rng_state = rng_state
        else:
            eng.set_seed(0 if seed is None else seed)
        res = eng.run_markov_chain(verbose=verbose, m=m, iterations=iterations, L=L, c_i=c_i, burnin=burnin,
                                   t=t, r=r, neal8=neal8, split_merge=split_merge, n8_step_size=n8_step_size,
                                   sam_step_size=sam_step_size, thinning=thinning, keep_params=keep_params)
        res["rng_state"] = eng.rng_state
        res["stats"] = eng.stats()
        return res
    finally:
        eng.close()
