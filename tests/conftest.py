import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _built_native():
    from mpit_amd import _build

    _build.build()
    yield


def has_gpu() -> bool:
    import torch

    return torch.cuda.is_available()
