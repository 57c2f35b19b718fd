"""HIP beam-search decoder and edit distance / CER against the oracle
(tests/test_oracle.py pins the oracle: exhaustive-beam == exact argmax,
LabelSeq merge quirk, edit-distance KATs)."""
import numpy as np
import pytest
import torch

from oracle import ref_graph as G

pytestmark = pytest.mark.gpu


def _logits(rng, T, B, C, kind):
    if kind == "random":
        return (rng.standard_normal((T, B, C)) * 2).astype(np.float32)
    # peaky: what a trained recogniser emits -- one dominant class per frame
    x = (rng.standard_normal((T, B, C)) * 0.5).astype(np.float32)
    cls = rng.integers(0, C, (T, B))
    cls[rng.random((T, B)) < 0.5] = C - 1
    np.put_along_axis(x, cls[..., None], 6.0 + rng.random((T, B, 1)).astype(np.float32) * 2, axis=2)
    return x


@pytest.mark.parametrize("T,B,C,K,merge,top,kind", [
    (30, 6, 96, 16, True, 1, "random"),
    (40, 5, 96, 128, True, 1, "peaky"),
    (20, 4, 96, 128, False, 3, "random"),
    (24, 6, 12, 8, True, 2, "random"),
    (60, 4, 96, 16, False, 2, "peaky"),
])
def test_beam_matches_oracle(cuda, T, B, C, K, merge, top, kind):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(T * 7 + K)
    x = _logits(rng, T, B, C, kind)
    seq = rng.integers(1, T + 1, B).astype(np.int32)
    seq[0] = T
    if B > 3:
        seq[1], seq[2] = 0, 1
    paths, logp = G.ctc_beam_search_decode(x, seq, beam_width=K, top_paths=top, merge_repeated=merge)
    out, out_len, lp = Kn.ctc_beam_decode(torch.from_numpy(x).to(cuda), torch.from_numpy(seq).to(cuda), K, top,
                                          merge)
    out, out_len, lp = out.cpu().numpy(), out_len.cpu().numpy(), lp.cpu().numpy()
    for k in range(top):
        for b in range(B):
            n = int(out_len[k, b])
            assert list(out[k, b, :n]) == paths[k][b], (k, b)
            assert (out[k, b, n:] == -1).all()
    fin = np.isfinite(logp)
    assert (np.isfinite(lp) == fin).all()
    # float32 log-sum-exp chains over <= 60 frames vs the float64 oracle
    np.testing.assert_allclose(lp[fin], logp[fin], rtol=1e-4, atol=2e-3)


def test_beam_labelseq_merge_quirk(cuda):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    x = np.full((4, 1, 3), -8.0, np.float32)
    x[0, 0, 0] = x[1, 0, 1] = x[2, 0, 2] = x[3, 0, 1] = 8.0          # A B blank B
    xs, sl = torch.from_numpy(x).to(cuda), torch.tensor([4], dtype=torch.int32, device=cuda)
    out, n, _ = Kn.ctc_beam_decode(xs, sl, 8, 1, True)
    assert out[0, 0, :int(n[0, 0])].tolist() == [0, 1]
    out, n, _ = Kn.ctc_beam_decode(xs, sl, 8, 1, False)
    assert out[0, 0, :int(n[0, 0])].tolist() == [0, 1, 1]


def test_beam_exhaustive_equals_exact_ctc(cuda):
    """Beam wide enough to keep every prefix: top path score == -ctc_loss."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(11)
    x = (rng.standard_normal((5, 3, 3)) * 2).astype(np.float32)
    seq = np.array([5, 5, 4], np.int32)
    out, n, lp = Kn.ctc_beam_decode(torch.from_numpy(x).to(cuda), torch.from_numpy(seq).to(cuda), 64, 1, False)
    for b in range(3):
        lab = out[0, b, :int(n[0, b])].tolist()
        exact = -G.ctc_loss_single(x[:seq[b], b].astype(np.float64), lab, 2)[0]
        assert abs(float(lp[b, 0]) - exact) < 1e-4


def test_edit_distance_matches_oracle(cuda):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(5)
    B = 97
    hl = rng.integers(0, 300, B).astype(np.int32)
    ll = rng.integers(0, 257, B).astype(np.int32)
    hl[:4] = [0, 0, 5, 70]
    ll[:4] = [0, 9, 0, 256]
    S, L = int(hl.max()), 256
    hyp = np.full((B, S), -1, np.int64)
    lab = np.zeros((B, L), np.int32)
    truths, hyps = [], []
    for b in range(B):
        t = rng.integers(0, 6, ll[b])                     # small alphabet -> many matches
        h = t[:hl[b]].copy() if rng.random() < 0.5 and hl[b] <= ll[b] else rng.integers(0, 6, hl[b])
        h = np.concatenate([h, rng.integers(0, 6, hl[b] - len(h))]) if len(h) < hl[b] else h
        hyp[b, :hl[b]] = h
        lab[b, :ll[b]] = t
        hyps.append(list(h))
        truths.append(list(t))
    want = np.array([G.edit_distance(h, t) for h, t in zip(hyps, truths)])
    totals = torch.zeros(3, dtype=torch.int32, device=cuda)
    d = Kn.edit_distance(torch.from_numpy(hyp).to(cuda), torch.from_numpy(hl).to(cuda),
                         torch.from_numpy(lab).to(cuda), torch.from_numpy(ll).to(cuda), totals)
    assert (d.cpu().numpy() == want).all()
    assert totals.tolist() == [int(want.sum()), int((want > 0).sum()), int(ll.sum())]


def test_get_testing_matches_oracle(cuda):
    """test.py:75-104 scalars: loss, label_error (CER), sequence_error."""
    from cnn_lstm_ctc_ocr_amd import test as ev
    rng = np.random.default_rng(9)
    T, B, C = 30, 6, 96
    x = _logits(rng, T, B, C, "peaky")
    seq = np.full(B, T, np.int32)
    labels = [list(rng.integers(0, 95, int(rng.integers(1, 10)))) for _ in range(B)]
    labels[0] = G.ctc_beam_search_single(x[:, 0], 128)[0][0] or [3]          # one exact hit
    loss, cer, serr = ev._get_testing(torch.from_numpy(x).to(cuda), torch.from_numpy(seq).to(cuda), labels)
    want_loss = np.mean([G.ctc_loss_single(x[:, b].astype(np.float64), labels[b], C - 1)[0] for b in range(B)])
    paths, _ = G.ctc_beam_search_decode(x, seq, beam_width=128)
    want_cer, want_serr = G.label_and_sequence_error(paths[0], labels)
    assert abs(float(loss) - want_loss) < 1e-3 * max(1.0, abs(want_loss))
    assert abs(float(cer) - want_cer) < 1e-6
    assert abs(float(serr) - want_serr) < 1e-6


def test_edit_distance_all_empty_decodes(cuda):
    """A batch whose decodes are all empty (an untrained model emitting only
    blanks) has a 0-column hypothesis tensor: the distance is each label's
    length, as tf.edit_distance(normalize=False) gives for an empty hypothesis."""
    from cnn_lstm_ctc_ocr_amd import decode
    hyp = torch.empty(3, 0, dtype=torch.int64, device=cuda)
    lab = torch.tensor([[1, 2, 3], [4, 0, 0], [0, 0, 0]], dtype=torch.int32, device=cuda)
    ln = torch.tensor([3, 1, 0], dtype=torch.int32, device=cuda)
    d = decode.edit_distance(hyp, torch.zeros(3, dtype=torch.int32, device=cuda), lab, ln)
    assert d.cpu().tolist() == [3.0, 1.0, 0.0]
