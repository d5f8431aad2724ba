import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi
    oracle_ffi.build()
    return oracle_ffi


@pytest.fixture(scope="session")
def zoo():
    from split_and_merge_gibbs_sampling_amd.data import load_zoo
    return load_zoo()
