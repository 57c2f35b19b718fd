"""The hipGraph-captured train step (train.GraphedStep) against the eager
train step: same kernels in the same order, so parameters, BatchNorm moving
statistics, Adam slots and losses must agree BIT FOR BIT over several steps
with a different batch loaded into the graph's static buffers each step; and
the graphed bf16 step at the bench shape (B=256, W=256, LSTM 512/512, the
ping-pong GEMM engines, persistent loops and side-stream paths included)
against the eager one."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batches(n, B, W, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        img = torch.from_numpy(rng.integers(0, 256, (B, 32, W, 1), dtype=np.uint8))
        widths = torch.from_numpy(rng.integers(W - 20, W + 1, B).astype(np.int32))
        lab = torch.from_numpy(rng.integers(0, 95, (B, 6)).astype(np.int32))
        ln = torch.from_numpy(rng.integers(1, 7, B).astype(np.int32))
        out.append((img, widths, lab, ln))
    return out


def _run(cuda, dtype, sizes, B, W, graphed, steps=3):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=sizes, dtype=dtype), device=cuda, seed=3)
    tr = Trainer(store)
    data = [(i.to(cuda), w.to(cuda), (lab.to(cuda), ln.to(cuda))) for i, w, lab, ln in _batches(steps, B, W, 7)]
    losses = []
    if graphed:
        g = tr.graphed(*data[0])
        for img, w, lab in data:
            losses.append(g.step(img, w, lab).item())
    else:
        for img, w, lab in data:
            losses.append(tr.step(img, w, lab).item())
    torch.cuda.synchronize()
    return losses, store.flat.cpu(), store.flat_stats.cpu(), tr.m.cpu(), tr.v.cpu(), tr.global_step


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_graphed_step_matches_eager_bitwise(cuda, dtype):
    sizes = (64, 64) if dtype == torch.float32 else (256, 256)     # bf16 step kernels tile H by 256
    a = _run(cuda, dtype, sizes, 64, 96, graphed=False)
    b = _run(cuda, dtype, sizes, 64, 96, graphed=True)
    assert a[0] == b[0]
    for x, y in zip(a[1:5], b[1:5]):
        assert torch.equal(x, y)
    assert a[5] == b[5] == 3


def test_graphed_step_bench_shape(cuda):
    a = _run(cuda, torch.bfloat16, (512, 512), 256, 256, graphed=False, steps=2)
    b = _run(cuda, torch.bfloat16, (512, 512), 256, 256, graphed=True, steps=2)
    assert np.allclose(a[0], b[0], rtol=1e-6), (a[0], b[0])
    assert torch.equal(a[1], b[1])


def test_graphed_step_rejects_other_shapes(cuda):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(64, 64), dtype=torch.float32), device=cuda, seed=0)
    img, w, lab, ln = _batches(1, 32, 64, 1)[0]
    g = Trainer(store).graphed(img.to(cuda), w.to(cuda), (lab.to(cuda), ln.to(cuda)))
    with pytest.raises(ValueError):
        g.step(torch.zeros(32, 32, 96, 1, dtype=torch.uint8, device=cuda))
    with pytest.raises(ValueError):
        g.step(label=(torch.zeros(32, 9, dtype=torch.int32, device=cuda), ln.to(cuda)))
