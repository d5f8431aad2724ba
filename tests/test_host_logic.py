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
