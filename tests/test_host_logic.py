"""Host-side logic of the engine that needs no GPU: the R stream generated ahead of
update_phi's serial draws (StreamAhead) and the split rbeta (csrc/rmath.hpp), compiled
with g++ from tests/cpp/host_rng_test.cpp."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_stream_ahead_and_split_rbeta(tmp_path):
    exe = tmp_path / "host_rng_test"
    src = os.path.join(HERE, "cpp", "host_rng_test.cpp")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), src],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(r.stderr)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "host rng ok" in r.stdout


def test_glibc_exp_log_replicas_match_libm(tmp_path):
    """csrc/glibc_math.hpp (used by the device pool generator) equals the host libm's exp and
    log bit for bit: special values, the generator's argument shapes, random bit patterns."""
    exe = tmp_path / "glibc_math_test"
    src = os.path.join(HERE, "cpp", "glibc_math_test.cpp")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), src],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(r.stderr)
    r = subprocess.run([str(exe), "1500000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 exp mismatches, 0 log mismatches" in r.stdout


def test_pool_pipeline_model_matches_sequential_generator(tmp_path):
    """The stream-exact pool pipeline (packed attempt tables -> host walk -> values; the
    arithmetic the device kernels share) reproduces the sequential generator's pool and
    stream position: Zoo hyperparameters at several stream offsets, odd D with an rbeta
    BC class, C3-like mixed levels, a C4-like 784-attribute run."""
    exe = tmp_path / "pool_gen_test"
    src = os.path.join(HERE, "cpp", "pool_gen_test.cpp")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), src],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(r.stderr)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "pool pipeline ok" in r.stdout


def test_host_pool_home_domain_choice(tmp_path):
    """csrc/host_topology.hpp: the L3 domain a context's host pool is homed on (one pool per
    home, engine.cpp HostPool::for_home), on synthetic node topologies."""
    exe = tmp_path / "host_topology_test"
    src = os.path.join(HERE, "cpp", "host_topology_test.cpp")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), src], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(r.stderr)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host topology ok" in r.stdout
