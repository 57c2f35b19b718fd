"""HIP CTC loss / gradient / greedy decode against the oracle (tests/test_oracle.py pins it)."""
import numpy as np
import pytest
import torch

from oracle import ref_graph as G

pytestmark = pytest.mark.gpu


def _labels(rng, B, T, lo=0, hi=19):
    labels = []
    for _ in range(B):
        while True:
            L = int(rng.integers(lo, hi + 1))
            lab = list(rng.integers(0, 95, L))
            if G.ctc_required_time(lab) <= T:
                break
        labels.append(lab)
    return labels


def _dense(labels, B):
    Lmax = max([len(l) for l in labels] + [1])
    d = np.zeros((B, Lmax), np.int32)
    for i, l in enumerate(labels):
        d[i, :len(l)] = l
    return d, np.array([len(l) for l in labels], np.int32)


@pytest.mark.parametrize("T,B,relu", [(125, 16, True), (61, 5, False), (30, 7, True)])
def test_ctc_loss_matches_oracle(cuda, T, B, relu):
    from cnn_lstm_ctc_ocr_amd import kernels as K
    rng = np.random.default_rng(T + B)
    logits = rng.standard_normal((T, B, 96)).astype(np.float32) * 3
    if relu:
        logits = np.maximum(logits, 0)
    seq = rng.integers(max(1, T // 2), T + 1, B).astype(np.int32)
    seq[0] = T
    labels = _labels(rng, B, int(seq.min()), lo=0, hi=min(19, int(seq.min()) // 2))
    lab, lablen = _dense(labels, B)
    ref_loss, ref_grad = G.ctc_loss(logits, labels, seq)
    loss, grad, status = K.ctc_loss(torch.from_numpy(logits).to(cuda), torch.from_numpy(lab).to(cuda),
                                    torch.from_numpy(lablen).to(cuda), torch.from_numpy(seq).to(cuda),
                                    grad_scale=0.5)
    assert status.cpu().sum().item() == 0
    # north_star tolerance: CTC loss within 1e-3 relative (fp32)
    np.testing.assert_allclose(loss.cpu().numpy(), ref_loss, rtol=1e-3)
    # fp32 log-space lattice: |grad| <= 1, abs error grows with -log p (~800 nats here)
    np.testing.assert_allclose(grad.cpu().numpy(), 0.5 * ref_grad, rtol=1e-3, atol=2e-4)


def test_ctc_long_labels_multi_register(cuda):
    """S = 2L+1 > 64 exercises the cross-register lattice shifts."""
    from cnn_lstm_ctc_ocr_amd import kernels as K
    rng = np.random.default_rng(3)
    T, B = 253, 3
    logits = rng.standard_normal((T, B, 96)).astype(np.float32)
    seq = np.array([253, 240, 200], np.int32)
    labels = [list(rng.integers(0, 95, 90)), [5] * 40 + [6] * 30, list(rng.integers(0, 95, 33))]
    lab, lablen = _dense(labels, B)
    ref_loss, ref_grad = G.ctc_loss(logits, labels, seq)
    loss, grad, _ = K.ctc_loss(torch.from_numpy(logits).to(cuda), torch.from_numpy(lab).to(cuda),
                               torch.from_numpy(lablen).to(cuda), torch.from_numpy(seq).to(cuda))
    np.testing.assert_allclose(loss.cpu().numpy(), ref_loss, rtol=1e-3)
    np.testing.assert_allclose(grad.cpu().numpy(), ref_grad, rtol=1e-3, atol=2e-4)


def test_ctc_infeasible_flags(cuda):
    from cnn_lstm_ctc_ocr_amd import _lib
    from cnn_lstm_ctc_ocr_amd import kernels as K
    K.status_word(cuda).zero_()
    logits = torch.zeros(3, 2, 96, device=cuda)
    lab = torch.tensor([[1, 1, 2], [1, 2, 3]], dtype=torch.int32, device=cuda)
    loss, grad, status = K.ctc_loss(logits, lab, torch.tensor([3, 3], dtype=torch.int32, device=cuda),
                                    torch.tensor([3, 3], dtype=torch.int32, device=cuda))
    assert status.cpu().tolist() == [1, 0]
    assert np.isinf(loss[0].item()) and np.isfinite(loss[1].item())
    assert K.read_status(cuda) == _lib.STATUS_CTC_INFEASIBLE
    assert K.read_status(cuda) == 0                        # read_status cleared it


def test_ctc_bad_lengths_and_labels_are_flagged_not_read(cuda):
    """label_len outside [0, max_label_len] or label values outside
    [0, C-1) must never index past the label row / the lattice: the row is
    flagged (status 2 / 3, loss +inf, zero gradient), the others are scored."""
    from cnn_lstm_ctc_ocr_amd import _lib
    from cnn_lstm_ctc_ocr_amd import kernels as K
    K.status_word(cuda).zero_()
    rng = np.random.default_rng(5)
    T, B, C = 20, 5, 96
    logits = torch.from_numpy(rng.standard_normal((T, B, C)).astype(np.float32)).to(cuda)
    lab = torch.tensor([[1, 2, 3], [1, 2, 3], [1, 95, 3], [4, -1, 3], [7, 8, 9]], dtype=torch.int32, device=cuda)
    ln = torch.tensor([3, 400, 3, 3, -2], dtype=torch.int32, device=cuda)
    seq = torch.full((B,), T, dtype=torch.int32, device=cuda)
    loss, grad, status = K.ctc_loss(logits, lab, ln, seq)
    assert status.cpu().tolist() == [0, 2, 3, 3, 2]
    lv = loss.cpu().numpy()
    assert np.isfinite(lv[0]) and np.all(np.isinf(lv[1:]))
    g = grad.cpu().numpy()
    assert np.all(g[:, 1:] == 0) and np.abs(g[:, 0]).sum() > 0
    ref_loss, _ = G.ctc_loss(logits.cpu().numpy()[:, :1], [[1, 2, 3]], np.array([T], np.int32))
    np.testing.assert_allclose(lv[0], ref_loss[0], rtol=1e-3)
    w = K.read_status(cuda)
    assert w == _lib.STATUS_CTC_BAD_LENGTH | _lib.STATUS_CTC_BAD_LABEL
    with pytest.raises(_lib.InvalidArgumentError):
        _lib.raise_for_status(w)


@pytest.mark.parametrize("merge", [True, False])
def test_greedy_decode_bit_exact(cuda, merge):
    from cnn_lstm_ctc_ocr_amd import kernels as K
    rng = np.random.default_rng(11)
    T, B = 125, 64
    # ReLU'd and quantised logits: many exact ties, exercising first-max
    logits = np.maximum(np.round(rng.standard_normal((T, B, 96)) * 2) / 2, 0).astype(np.float32)
    logits[:, :, 95] += (rng.random((T, B)) < 0.5) * 3.0        # frequent blanks
    seq = rng.integers(1, T + 1, B).astype(np.int32)
    ref, ref_neg = G.ctc_greedy_decode(logits, seq, merge_repeated=merge)
    out, out_len, neg = K.ctc_greedy_decode(torch.from_numpy(logits).to(cuda),
                                            torch.from_numpy(seq).to(cuda), merge)
    out, out_len = out.cpu().numpy(), out_len.cpu().numpy()
    for b in range(B):
        assert out_len[b] == len(ref[b])
        assert out[b, :out_len[b]].tolist() == ref[b]
        assert np.all(out[b, out_len[b]:] == -1)
    np.testing.assert_allclose(neg.cpu().numpy(), ref_neg, rtol=1e-6)
