import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE_DATA = "/root/reference/data"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libocrk.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU (run with -m 'not gpu' on CPU hosts)")
    return torch.device("cuda:0")
