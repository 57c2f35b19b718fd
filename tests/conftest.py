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


class _Opts:
    """Engine options set by a test, restored at teardown (cnn_lstm_ctc_ocr_amd.options)."""

    def __init__(self):
        self.saved = []

    def __call__(self, name, value):
        from cnn_lstm_ctc_ocr_amd import options
        self.saved.append((name, options.set(name, value)))

    def reset(self, name):
        """Back to the value the option had before this test first set it."""
        from cnn_lstm_ctc_ocr_amd import options
        for n, v in self.saved:
            if n == name:
                options.set(n, v)
                return

    def restore(self):
        from cnn_lstm_ctc_ocr_amd import options
        for n, v in reversed(self.saved):
            options.set(n, v)
        self.saved.clear()


@pytest.fixture
def ocrk_opts():
    o = _Opts()
    yield o
    o.restore()
