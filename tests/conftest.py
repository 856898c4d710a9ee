import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs through the C-ABI")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu_device():
    if not has_gpu():
        pytest.fail("GPU test collected on a machine without a GPU (run with -m 'not gpu')")
    return 0
