import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvectorwave_amd.so on cuda:0)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def engine():
    # a `-m gpu` run on a box whose GPU is not visible must FAIL, not pass with every parity check skipped
    if not gpu_available():
        pytest.fail("no GPU visible: the -m gpu parity tests need an MI355X (cuda:0)")
    from vectorwave_amd import Engine
    return Engine.get(0)
