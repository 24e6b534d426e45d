import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "ceres-solver-cuda_amd"), os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libcse.so on HIP)")
    config.addinivalue_line("markers", "slow: full-size (BAL problem-13682) checks")


@pytest.fixture(scope="session")
def gpu():
    """Skip-free guard: -m gpu tests require a GPU and the built library."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    from ceres_amd import _cse
    _cse.lib()
    return torch.device("cuda:0")
