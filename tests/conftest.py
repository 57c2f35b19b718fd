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


@pytest.fixture(scope="session")
def trained_fp32(cuda):
    """The LSTM 512/512 model trained in fp32 on the reference's data/val shard
    (tests/trained_model.py REGIME), once per session: shared by the trained-weight
    parity tests (test_gpu_trained*.py). Returns dict(store, losses, curves, state)."""
    import torch
    import trained_model as TM
    batches = TM.shard_batches(TM.TRAIN_SHARD)
    dev = TM.to_device(batches, cuda, torch.float32)
    from cnn_lstm_ctc_ocr_amd import model
    store, losses, curves = TM.train_on_shard(
        torch.float32, batches, cuda, evals={"infer": lambda s: TM.shard_cer(s, dev),
                                             "train_mode": lambda s: TM.shard_cer(s, dev, model.TRAIN)})
    return {"store": store, "losses": losses, "curves": curves, "state": store.state_dict(), "batches": batches}


@pytest.fixture(scope="session")
def trained_bf16(cuda, trained_fp32):
    """The same run in bf16 (the benched precision)."""
    import torch
    import trained_model as TM
    batches = trained_fp32["batches"]
    dev = TM.to_device(batches, cuda, torch.bfloat16)
    store, losses, curves = TM.train_on_shard(torch.bfloat16, batches, cuda,
                                              evals={"infer": lambda s: TM.shard_cer(s, dev)})
    return {"store": store, "losses": losses, "curves": curves}
