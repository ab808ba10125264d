import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="session")
def cuda_device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    return torch.device("cuda:0")


@pytest.fixture
def launch_policy():
    """Set fields of the library's launch policy (swh_set_launch_policy) for one
    test; the policy in force before the first call is restored afterwards."""
    from swh_trl_amd import _lib
    saved = []

    def set_(**fields):
        old = _lib.set_launch_policy(**fields)
        if not saved:
            saved.append(old)

    yield set_
    if saved:
        _lib.set_launch_policy(**saved[0])
