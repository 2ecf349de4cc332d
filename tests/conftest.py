import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import dtg  # noqa: E402,F401  (registers the `dtg` package)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the gfx950 HIP kernels)")
    config.addinivalue_line("markers", "slow: multi-process / long CPU tests")


@pytest.fixture
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
