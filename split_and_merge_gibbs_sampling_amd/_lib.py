"""ctypes binding of libhdpm.so (include/hdpm.h).

The shared library is built in-tree (split_and_merge_gibbs_sampling_amd/libhdpm.so) by
``build()``.  There is no CPU fallback: loading fails loudly if the library is missing,
and creating an engine fails loudly if no gfx950 device is visible.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libhdpm.so")
# A/B builds of the same library (tools/ab_*.sh): HDPM_LIB_VARIANT=x loads libhdpm_x.so
if os.environ.get("HDPM_LIB_VARIANT"):
    LIB_PATH = os.path.join(PKG_DIR, f"libhdpm_{os.environ['HDPM_LIB_VARIANT']}.so")
CSRC = os.path.join(PKG_DIR, "csrc")

EXPORTS = (
    "hdpm_device_count", "hdpm_ctx_create", "hdpm_ctx_destroy", "hdpm_last_error", "hdpm_set_data",
    "hdpm_rng_set_seed", "hdpm_rng_set_state", "hdpm_rng_get_state", "hdpm_set_state", "hdpm_get_state",
    "hdpm_set_pool", "hdpm_get_pool", "hdpm_generate_pool", "hdpm_neal8_sweep", "hdpm_update_phi",
    "hdpm_compute_loglikelihood", "hdpm_loglik_matrix", "hdpm_restricted_gibbs", "hdpm_logprobgs_c_i",
    "hdpm_split_and_merge", "hdpm_run_markov_chain", "hdpm_get_stats", "hdpm_reset_stats",
    "hdpm_set_debug", "hdpm_synchronize", "hdpm_drop_prepared", "hdpm_init_chain", "hdpm_iteration", "hdpm_iterations", "hdpm_iterations_record", "hdpm_record_take", "hdpm_rng_fill_device",
    "hdpm_get_pool_heads", "hdpm_set_option", "hdpm_get_option", "hdpm_debug_draw", "hdpm_debug_math",
    "hdpm_psm_build", "hdpm_psm_rows", "hdpm_psm_vi_lb",
)

OPT_HIG_LOGSPACE = 1
OPT_PHI_DEVICE = 2
OPT_PIPE_WAIT_US = 3
OPT_FPG_WAIT_US = 4
OPT_FPG_FAIL_AT = 5
OPT_EXACT_KERNEL = 6
OPT_LAT_NEGLIGIBLE = 7
OPT_SM_WIDE_WAIT_US = 8
OPT_SM_CHAIN = 9

STATUS = {0: "OK", 1: "E_VALIDATE", 2: "E_GSL", 3: "E_PROB", 4: "E_WALKER", 5: "E_ARG",
          6: "E_DEVICE", 7: "E_NODEVICE"}


class HdpmError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"hdpm {STATUS.get(status, status)}: {msg}")
        self.status = status


class ChainParams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "verbose", "m", "iterations", "L", "burnin", "t", "r", "neal8", "split_merge",
        "n8_step_size", "sam_step_size", "thinning")]


class Stats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "sweeps", "rounds", "restarts", "exact_points", "moves", "checked_rounds", "prepass_points")] + \
        [(n, C.c_double) for n in (
            "t_prepass_ms", "t_resolve_ms", "t_stats_ms", "t_host_phi_ms", "t_rng_ms", "t_loglik_ms",
            "t_exact_ms")] + \
        [(n, C.c_int64) for n in ("pool_calls", "pool_entries", "pool_device_calls")] + \
        [(n, C.c_double) for n in (
            "t_pool_ms", "t_pool_mt_ms", "t_pool_accept_ms", "t_pool_parse_ms", "t_pool_values_ms")] + \
        [(n, C.c_int64) for n in ("phi_spec_runs", "phi_spec_clusters", "prepass_timed", "prepass_timed_points",
                                  "rng_windows", "rng_windows_fresh", "listed_points", "sm_moves")] + \
        [(n, C.c_double) for n in ("t_sm_ms", "t_sm_scan_ms", "t_sm_phi_ms", "t_sm_terms_ms")] + \
        [(n, C.c_int64) for n in ("phi_device_calls", "phi_device_fallbacks", "phi_device_last_status",
                                  "phi_lookahead_hits", "phi_lookahead_copies", "pipe_enqueued", "pipe_runs",
                                  "pipe_refused", "pipe_recovered", "phi_tree_calls", "phi_tree_retries",
                                  "pool_walk_fallbacks", "phi_dspec_launched", "phi_dspec_used",
                                  "fpg_launches", "phi_sm_device_calls", "phi_fallback_status_mask",
                                  "phi_sm_window_retries", "fpg_aborts", "exact_mass_launches",
                                  "exact_lanes_launches", "dense_launches", "sm_wide_scans",
                                  "sm_wide_fallbacks", "phi_fast_calls", "phi_fast_handbacks",
                                  "labels_mirrored", "labels_downloaded", "phi_state_direct",
                                  "phi_chain_launched", "phi_chain_used", "phi_chain_dropped",
                                  "pipe_auto", "pipe_desync", "sm_chain_runs", "sm_chain_scans",
                                  "sm_chain_resumes")]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def build(force: bool = False) -> str:
    """Compile the HIP kernels + host runtime for gfx950 into LIB_PATH (hipcc)."""
    srcs = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    stale = force or not os.path.exists(LIB_PATH) or \
        max(os.path.getmtime(s) for s in srcs) > os.path.getmtime(LIB_PATH)
    if stale:
        subprocess.run(["make", "-s", "-C", CSRC], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libhdpm.so not built ({LIB_PATH}); run __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, f64 = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    P = C.POINTER
    sig = {
        "hdpm_device_count": ([], C.c_int),
        "hdpm_ctx_create": ([i32, P(vp)], C.c_int),
        "hdpm_ctx_destroy": ([vp], None),
        "hdpm_last_error": ([vp], C.c_char_p),
        "hdpm_set_data": ([vp, vp, i32, i32, vp, f64, vp, vp], C.c_int),
        "hdpm_rng_set_seed": ([vp, C.c_uint32], C.c_int),
        "hdpm_rng_set_state": ([vp, vp], C.c_int),
        "hdpm_rng_get_state": ([vp, vp], C.c_int),
        "hdpm_set_state": ([vp, vp, i32, vp, vp], C.c_int),
        "hdpm_get_state": ([vp, vp, P(i32), vp, vp, i32], C.c_int),
        "hdpm_set_pool": ([vp, vp, vp, i64], C.c_int),
        "hdpm_get_pool": ([vp, vp, vp, i64], C.c_int),
        "hdpm_generate_pool": ([vp, i64], C.c_int),
        "hdpm_neal8_sweep": ([vp, i32], C.c_int),
        "hdpm_update_phi": ([vp, vp, i32], C.c_int),
        "hdpm_compute_loglikelihood": ([vp, P(f64)], C.c_int),
        "hdpm_loglik_matrix": ([vp, vp, vp], C.c_int),
        "hdpm_restricted_gibbs": ([vp, vp, i32, i32, i32, i32], C.c_int),
        "hdpm_logprobgs_c_i": ([vp, vp, vp, i32, i32, i32, P(f64)], C.c_int),
        "hdpm_split_and_merge": ([vp, i32, i32, i32, P(i32)], C.c_int),
        "hdpm_run_markov_chain": ([vp, P(ChainParams), vp, vp, vp, vp, vp, vp, vp], C.c_int),
        "hdpm_get_stats": ([vp, P(Stats)], C.c_int),
        "hdpm_init_chain": ([vp, P(ChainParams), vp], C.c_int),
        "hdpm_iteration": ([vp, P(ChainParams), i32, P(i32), P(i32), P(f64)], C.c_int),
        "hdpm_iterations": ([vp, P(ChainParams), i32, i32, P(i32), vp, vp], C.c_int),
        "hdpm_iterations_record": ([vp, P(ChainParams), i32, i32, P(i32), vp, vp, vp, vp, P(i32)], C.c_int),
        "hdpm_record_take": ([vp, vp, vp, P(i64)], C.c_int),
        "hdpm_reset_stats": ([vp], C.c_int),
        "hdpm_rng_fill_device": ([vp, i64, vp], C.c_int),
        "hdpm_set_debug": ([vp, i32], C.c_int),
        "hdpm_synchronize": ([vp], C.c_int),
        "hdpm_drop_prepared": ([vp], C.c_int),
        "hdpm_get_pool_heads": ([vp, vp, i64], C.c_int),
        "hdpm_set_option": ([vp, i32, f64], C.c_int),
        "hdpm_get_option": ([vp, i32, P(f64)], C.c_int),
        "hdpm_debug_draw": ([vp, vp, i32, f64, i32, i32, P(i32)], C.c_int),
        "hdpm_debug_math": ([vp, vp, i64, i32, i32, vp], C.c_int),
        "hdpm_psm_build": ([vp, vp, i32, i32], C.c_int),
        "hdpm_psm_rows": ([vp, i32, i32, vp], C.c_int),
        "hdpm_psm_vi_lb": ([vp, vp, i32, vp], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)
