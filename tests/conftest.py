import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import __graft_entry__  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def pkg():
    return __graft_entry__.load_package()


@pytest.fixture(scope="session")
def O():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def ctx(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg.Context(0)
