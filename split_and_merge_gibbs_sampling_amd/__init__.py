"""MI355X-native Neal-8 / split-merge reassignment engine for Hamming-kernel DP mixtures.

Drop-in for the hot path of Filippo-Galli/Split_and_merge_Gibbs_sampling: the gfx950
kernels and the host runtime live in ``libhdpm.so`` (C ABI: include/hdpm.h); this
package is the Python mirror of the reference interface.
"""
from ._lib import HdpmError, build  # noqa: F401
from .sampler import Engine, run_markov_chain  # noqa: F401

__all__ = ["Engine", "run_markov_chain", "HdpmError", "build"]
