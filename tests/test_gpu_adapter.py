"""The Rcpp adapter's call sequence on the MI355X.

integration/launcher_hip.cpp is the reference's R entry point run_markov_chain
(code/launcher.cpp:6-14) backed by libhdpm.so; its body, integration/hdpm_chain.hpp, has no
R types, and tests/cpp/adapter_replay.cpp (built by __graft_entry__.build into
integration/adapter_replay) runs it against the oracle's run_markov_chain (la:6-174) over
consecutive calls sharing one random stream: .Random.seed in (hdpm_rng_set_state) ->
hdpm_init_chain -> hdpm_iteration loop with hdpm_get_state at every saved iteration ->
hdpm_rng_get_state -> the next call.  Labels, K, acceptances, final_ass and the stream
after each call bit for bit, log-likelihoods within 1e-10 relative; `time` inside the call's
wall time (the clock starts after init_chain, la:79); non-integer or out-of-range doubles in
the data matrix rejected with HDPM_E_ARG before any narrowing cast.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "integration", "adapter_replay")


def write_spec(path, ds, seed, calls):
    with open(path, "wb") as f:
        f.write(struct.pack("<iid", ds.n, ds.d, float(ds.gamma)))
        f.write(np.ascontiguousarray(ds.attrisize, "<i4").tobytes())
        f.write(np.ascontiguousarray(ds.v, "<f8").tobytes())
        f.write(np.ascontiguousarray(ds.w, "<f8").tobytes())
        f.write(np.asfortranarray(ds.codes.astype("<f8")).tobytes(order="F"))
        f.write(struct.pack("<Ii", seed, len(calls)))
        for params, init in calls:
            f.write(np.array(params, "<i4").tobytes())
            f.write(struct.pack("<i", 0 if init is None else 1))
            if init is not None:
                f.write(np.ascontiguousarray(init, "<i4").tobytes())


def params(m=3, iterations=20, L=1, burnin=10, t=10, r=10, neal8=1, split_merge=1, n8=1, sam=1, thinning=1):
    return [0, m, iterations, L, burnin, t, r, neal8, split_merge, n8, sam, thinning]


def run(tmp_path, ds, seed, calls):
    assert os.path.exists(BIN), "integration/adapter_replay not built (__graft_entry__.build)"
    spec = os.path.join(tmp_path, "spec.bin")
    write_spec(spec, ds, seed, calls)
    r = subprocess.run([BIN, spec], capture_output=True, text=True, timeout=600)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("match") == len(calls)
    # poisoned NumericMatrix values (1.5, 257, 0, -1, NaN, m_j + 1) are rejected before the cast
    assert r.stdout.count("rejected") == 6


def test_adapter_zoo_consecutive_calls(tmp_path, zoo):
    # zoo_simulator.R:138-155 shapes: L = 1 from all-zero labels, then a random init with
    # thinning, then Neal-8 only -- three calls on one stream, no set.seed in between
    calls = [(params(m=3, iterations=30, L=1, burnin=20, neal8=1, split_merge=1), np.zeros(zoo.n, np.int32)),
             (params(m=3, iterations=15, L=1, burnin=5, thinning=2, neal8=1, split_merge=1), None),
             (params(m=2, iterations=25, L=1, burnin=0, neal8=1, split_merge=0), zoo.truth)]
    run(str(tmp_path), zoo, 1, calls)


def test_adapter_synthetic_split_merge_steps(tmp_path):
    from split_and_merge_gibbs_sampling_amd.data import hamming_mixture
    ds = hamming_mixture(3000, 24, 6, (2, 5), seed=17)
    calls = [(params(m=3, iterations=8, L=1, burnin=2, n8=2, sam=3, neal8=1, split_merge=1), ds.truth),
             (params(m=3, iterations=6, L=1, burnin=0, neal8=1, split_merge=0), None)]
    run(str(tmp_path), ds, 7, calls)
