import os
import sys

import pytest

# every HIP launch in the GPU tier is checked and synchronised by the op that
# issued it (csrc/bindings.cpp check_launch), so a fault names its kernel
os.environ.setdefault("MCP_CHECK_LAUNCH", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels, RCCL)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def gpu_available():
    import torch
    return torch.cuda.is_available()
