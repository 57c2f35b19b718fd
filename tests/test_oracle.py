"""Pin the CPU oracle (oracle/) before trusting it as the parity checker.

Sources of truth, in order: the reference's own fixture data (TFRecord shards
under /root/reference/data, when present), known-answer tests (brute-force CTC
path sums, hand-made greedy cases, finite differences), and independent
PyTorch-CPU implementations where TF1 semantics coincide.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_graph as G
from oracle import ref_model as M

from conftest import REFERENCE_DATA

torch.set_num_threads(min(8, os.cpu_count() or 1))


def _nchw(x):
    return torch.from_numpy(np.ascontiguousarray(x.transpose(0, 3, 1, 2)))


def _nhwc(t):
    return t.detach().numpy().transpose(0, 2, 3, 1)


# ------------------------------------------------------------ charset / data
def test_charset_constants():
    assert G.NUM_CLASSES == 95 and G.BLANK == 95
    assert G.OUT_CHARSET[:3] == "ABC" and G.OUT_CHARSET[62] == " "
    assert G.encode_text("MONIKER") == [12, 14, 13, 8, 10, 4, 17]   # mjsynth-tfrecord.py:149-150
    assert G.get_string([12, 14, 13, 8, 10, 4, 17]) == "MONIKER"


@pytest.mark.skipif(not os.path.isdir(REFERENCE_DATA), reason="reference data not mounted")
def test_reference_tfrecords_pin_label_encoding():
    """Every record of the reference's own shards: labels == encode(text)."""
    from cnn_lstm_ctc_ocr_amd.tfrecord import read_word_records
    n = 0
    for split in ("test", "val"):
        for r in read_word_records(os.path.join(REFERENCE_DATA, split, "words-000.tfrecord"),
                                   verify_crc=True):
            assert r["labels"] == G.encode_text(r["text"])
            assert r["length"] == len(r["text"])
            n += 1
    assert n == 892 + 803


def test_seq_len():
    assert list(G.seq_len_from_width([128, 256, 512, 33])) == [61, 125, 253, 13]


def test_preprocess_values():
    x = np.arange(256, dtype=np.uint8)
    y = G.preprocess(x)
    assert y.dtype == np.float32
    assert y[0] == np.float32(-0.5) and y[255] == np.float32(255) * np.float32(1 / 255.) - np.float32(0.5)
    t = G.preprocess_train(np.zeros((31, 5, 1), np.uint8))
    assert t.shape == (32, 5, 1)


# ------------------------------------------------------------------ conv/pool
@pytest.mark.parametrize("pad", ["same", "valid"])
def test_conv2d_vs_torch(pad):
    rng = np.random.default_rng(1)
    x = rng.standard_normal((2, 7, 9, 4))
    w = rng.standard_normal((3, 3, 4, 5))
    b = rng.standard_normal(5)
    y = G.conv2d(x, w, b, pad)
    xt = _nchw(x).requires_grad_()
    wt = torch.from_numpy(w.transpose(3, 2, 0, 1).copy()).requires_grad_()
    bt = torch.from_numpy(b).requires_grad_()
    yt = F.conv2d(xt, wt, bt, padding=1 if pad == "same" else 0)
    np.testing.assert_allclose(y, _nhwc(yt), rtol=1e-10, atol=1e-10)
    dy = rng.standard_normal(y.shape)
    yt.backward(_nchw(dy))
    dx, dw, db = G.conv2d_bwd(x, w, dy, pad)
    np.testing.assert_allclose(dx, _nhwc(xt.grad), rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(dw, wt.grad.numpy().transpose(2, 3, 1, 0), rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(db, bt.grad.numpy(), rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("pool", [(2, 2, 2, 2), (2, 2, 2, 1), (3, 1, 3, 1)])
def test_maxpool_vs_torch(pool):
    kh, kw, sh, sw = pool
    rng = np.random.default_rng(2)
    x = rng.standard_normal((2, 7, 9, 3))
    y = G.maxpool(x, *pool)
    xt = _nchw(x).requires_grad_()
    yt = F.max_pool2d(xt, (kh, kw), (sh, sw))
    np.testing.assert_array_equal(y, _nhwc(yt))
    dy = rng.standard_normal(y.shape)
    yt.backward(_nchw(dy))
    np.testing.assert_allclose(G.maxpool_bwd(x, dy, *pool), _nhwc(xt.grad), rtol=1e-12, atol=1e-12)


def test_maxpool_bwd_first_max_tie():
    x = np.zeros((1, 2, 2, 1))
    dx = G.maxpool_bwd(x, np.ones((1, 1, 1, 1)), 2, 2, 2, 2)
    assert dx[0, 0, 0, 0] == 1 and dx.sum() == 1


def test_batchnorm_vs_torch():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((3, 4, 5, 6)) * 2 + 1
    g, b = rng.standard_normal(6), rng.standard_normal(6)
    y, mean, var, var_u, cache = G.bn_train(x, g, b)
    xt = _nchw(x).requires_grad_()
    gt, bt = torch.from_numpy(g).requires_grad_(), torch.from_numpy(b).requires_grad_()
    rm, rv = torch.zeros(6, dtype=torch.float64), torch.ones(6, dtype=torch.float64)
    yt = F.batch_norm(xt, rm, rv, gt, bt, training=True, momentum=0.01, eps=1e-3)
    np.testing.assert_allclose(y, _nhwc(yt), rtol=1e-10, atol=1e-10)
    # torch's running_var uses the unbiased batch variance, as TF1's fused BN does
    np.testing.assert_allclose(G.bn_moving_update(np.ones(6), var_u), rv.numpy(), rtol=1e-10)
    np.testing.assert_allclose(G.bn_moving_update(np.zeros(6), mean), rm.numpy(), rtol=1e-10)
    dy = rng.standard_normal(y.shape)
    yt.backward(_nchw(dy))
    dx, dg, db = G.bn_bwd(dy, cache, g)
    np.testing.assert_allclose(dx, _nhwc(xt.grad), rtol=1e-9, atol=1e-10)
    np.testing.assert_allclose(dg, gt.grad.numpy(), rtol=1e-9)
    np.testing.assert_allclose(db, bt.grad.numpy(), rtol=1e-9)


# ----------------------------------------------------------------- LSTM / GRU
def _torch_lstm_from_tf(kernel, bias, n_in):
    """TF [i, j, f, o] kernel [In+H, 4H] -> torch nn.LSTM (gates i, f, g, o), f-bias +1."""
    H = kernel.shape[1] // 4
    i, j, f, o = np.split(kernel, 4, axis=1)
    bi, bj, bf, bo = np.split(bias, 4)
    wt = np.concatenate([i, f, j, o], axis=1)
    bt = np.concatenate([bi, bf + 1.0, bj, bo])
    lstm = torch.nn.LSTM(n_in, H, dtype=torch.float64)
    with torch.no_grad():
        lstm.weight_ih_l0.copy_(torch.from_numpy(wt[:n_in].T.copy()))
        lstm.weight_hh_l0.copy_(torch.from_numpy(wt[n_in:].T.copy()))
        lstm.bias_ih_l0.copy_(torch.from_numpy(bt))
        lstm.bias_hh_l0.zero_()
    return lstm


def test_lstm_direction_vs_torch_lstm():
    rng = np.random.default_rng(4)
    T, B, n_in, H = 6, 3, 5, 4
    x = rng.standard_normal((T, B, n_in))
    k = rng.standard_normal((n_in + H, 4 * H)) * 0.5
    b = rng.standard_normal(4 * H) * 0.5
    seq = np.array([6, 4, 1])
    lstm = _torch_lstm_from_tf(k, b, n_in)
    out_fw, _ = G.lstm_dir_fwd(x, seq, k, b, reverse=False)
    out_bw, _ = G.lstm_dir_fwd(x, seq, k, b, reverse=True)
    for bi in range(B):
        L = seq[bi]
        xt = torch.from_numpy(x[:L, bi:bi + 1])
        ref_fw = lstm(xt)[0][:, 0].detach().numpy()
        ref_bw = lstm(torch.flip(xt, [0]))[0][:, 0].detach().numpy()[::-1]
        np.testing.assert_allclose(out_fw[:L, bi], ref_fw, rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(out_bw[:L, bi], ref_bw, rtol=1e-10, atol=1e-12)
        assert np.all(out_fw[L:, bi] == 0) and np.all(out_bw[L:, bi] == 0)


def _torch_dir(x, seq, params, reverse, cell):
    """Autograd restatement of one dynamic_rnn direction in torch ops."""
    T, B, _ = x.shape
    rows = torch.arange(B)
    seq_t = torch.from_numpy(seq)
    if cell == "lstm":
        k, b = params
        H = k.shape[1] // 4
        c = torch.zeros(B, H, dtype=x.dtype)
    else:
        gk, gb, ck, cb = params
        H = ck.shape[1]
    h = torch.zeros(B, H, dtype=x.dtype)
    out = torch.zeros(T, B, H, dtype=x.dtype)
    for s in range(T):
        valid = (s < seq_t)[:, None]
        t_idx = torch.full((B,), s) if not reverse else torch.where(s < seq_t, seq_t - 1 - s, torch.full((B,), s))
        xs = x[t_idx, rows]
        if cell == "lstm":
            i, j, f, o = torch.split(torch.cat([xs, h], 1) @ k + b, H, 1)
            c_new = torch.sigmoid(f + 1.0) * c + torch.sigmoid(i) * torch.tanh(j)
            h_new = torch.sigmoid(o) * torch.tanh(c_new)
            c = torch.where(valid, c_new, c)
        else:
            r, u = torch.split(torch.sigmoid(torch.cat([xs, h], 1) @ gk + gb), H, 1)
            cand = torch.tanh(torch.cat([xs, r * h], 1) @ ck + cb)
            h_new = u * h + (1 - u) * cand
        out = out.index_put((t_idx, rows), torch.where(valid, h_new, out[t_idx, rows]))
        h = torch.where(valid, h_new, h)
    return out


@pytest.mark.parametrize("cell", ["lstm", "gru"])
@pytest.mark.parametrize("reverse", [False, True])
def test_rnn_direction_backward_vs_autograd(cell, reverse):
    rng = np.random.default_rng(5)
    T, B, n_in, H = 5, 3, 4, 3
    x = rng.standard_normal((T, B, n_in))
    seq = np.array([5, 3, 2])
    if cell == "lstm":
        params = [rng.standard_normal((n_in + H, 4 * H)) * 0.5, rng.standard_normal(4 * H) * 0.5]
        out, cache = G.lstm_dir_fwd(x, seq, *params, reverse)
    else:
        params = [rng.standard_normal((n_in + H, 2 * H)) * 0.5, rng.standard_normal(2 * H) * 0.5,
                  rng.standard_normal((n_in + H, H)) * 0.5, rng.standard_normal(H) * 0.5]
        out, cache = G.gru_dir_fwd(x, seq, *params, reverse)
    xt = torch.from_numpy(x).requires_grad_()
    pt = [torch.from_numpy(p).requires_grad_() for p in params]
    ot = _torch_dir(xt, seq, pt, reverse, cell)
    np.testing.assert_allclose(out, ot.detach().numpy(), rtol=1e-10, atol=1e-12)
    dout = rng.standard_normal(out.shape)
    ot.backward(torch.from_numpy(dout))
    if cell == "lstm":
        dx, dk, db = G.lstm_dir_bwd(dout, cache, params[0], n_in)
        grads = [dk, db]
    else:
        dx, dgk, dgb, dck, dcb = G.gru_dir_bwd(dout, cache, params[0], params[2], n_in)
        grads = [dgk, dgb, dck, dcb]
    np.testing.assert_allclose(dx, xt.grad.numpy(), rtol=1e-9, atol=1e-12)
    for g, p in zip(grads, pt):
        np.testing.assert_allclose(g, p.grad.numpy(), rtol=1e-9, atol=1e-12)


def test_gru_cell_reset_before_matmul_kat():
    """TF1 GRU: candidate uses (r*h) @ Wc_h, which differs from torch's r*(h @ W_hn)."""
    x = np.array([[1.0]])
    h = np.array([[2.0]])
    gk = np.zeros((2, 2))
    gb = np.array([0.0, 0.0])                    # r = u = 0.5
    ck = np.array([[0.0], [1.0]])
    cb = np.array([1.0])                         # cand = tanh(0.5*2*1 + 1) = tanh(2)
    h_new, (r, u, cand) = G.gru_cell(x, h, gk, gb, ck, cb)
    assert np.isclose(cand[0, 0], np.tanh(2.0))
    assert np.isclose(h_new[0, 0], 0.5 * 2.0 + 0.5 * np.tanh(2.0))


# ------------------------------------------------------------------------ CTC
@pytest.mark.parametrize("labels", [[0], [1, 2], [1, 1], [2, 0, 2], []])
def test_ctc_loss_bruteforce_kat(labels):
    rng = np.random.default_rng(6)
    T, C = 5, 4                                   # classes 0..2, blank 3
    logits = rng.standard_normal((T, C))
    loss, _ = G.ctc_loss_single(logits, labels, blank=3)
    np.testing.assert_allclose(loss, G.ctc_loss_bruteforce(logits, labels, blank=3), rtol=1e-12)


def test_ctc_loss_and_grad_vs_torch():
    rng = np.random.default_rng(7)
    T, B, C = 20, 4, 96
    logits = rng.standard_normal((T, B, C)) * 2
    seq = np.array([20, 17, 9, 12])
    labels = [list(rng.integers(0, 95, 6)), [3, 3, 3, 1], [5], list(rng.integers(0, 95, 5))]
    losses, grad = G.ctc_loss(logits, labels, seq)
    lt = torch.from_numpy(logits).requires_grad_()
    tgt = torch.tensor([v for l in labels for v in l], dtype=torch.long)
    ref = F.ctc_loss(F.log_softmax(lt, -1), tgt, torch.from_numpy(seq),
                     torch.tensor([len(l) for l in labels]), blank=95, reduction="none")
    np.testing.assert_allclose(losses, ref.detach().numpy(), rtol=1e-10)
    ref.sum().backward()
    np.testing.assert_allclose(grad, lt.grad.numpy(), rtol=1e-8, atol=1e-10)
    assert np.all(grad[9:, 2] == 0)


def test_ctc_infeasible_raises():
    with pytest.raises(G.InfeasibleLabelError):
        G.ctc_loss_single(np.zeros((3, 96)), [1, 1, 2])          # needs 4 frames
    G.ctc_loss_single(np.zeros((4, 96)), [1, 1, 2])              # exactly enough


# ------------------------------------------------------------- greedy decode
def test_greedy_decode_kat():
    C = 96
    seq_ids = [1, 1, 95, 1, 2, 2, 95, 95, 3]
    logits = np.zeros((len(seq_ids) + 2, 2, C), np.float32)
    for t, k in enumerate(seq_ids):
        logits[t, 0, k] = 1.0
    logits[:, 1, 7] = 2.0
    logits[:, 1, 9] = 2.0                         # tie -> first max (7)
    seqs, neg = G.ctc_greedy_decode(logits, np.array([len(seq_ids), 3]))
    assert seqs[0] == [1, 1, 2, 3]
    assert seqs[1] == [7]
    np.testing.assert_allclose(neg, [-len(seq_ids), -6.0])
    seqs_nm, _ = G.ctc_greedy_decode(logits, np.array([len(seq_ids), 3]), merge_repeated=False)
    assert seqs_nm[0] == [1, 1, 1, 2, 2, 3]
    dense = G.to_dense(seqs)
    assert dense.dtype == np.int64 and dense.tolist() == [[1, 1, 2, 3], [7, -1, -1, -1]]


def test_greedy_all_zero_logits_emit_label_zero():
    """ReLU logits are often all 0: argmax is class 0 ('A'), merged to one."""
    seqs, _ = G.ctc_greedy_decode(np.zeros((5, 1, 96), np.float32), np.array([5]))
    assert seqs == [[0]]


def _best_labeling(logits, blank):
    import itertools
    T, C = logits.shape
    best = None
    for L in range(T + 1):
        for lab in itertools.product([c for c in range(C) if c != blank], repeat=L):
            if G.ctc_required_time(lab) > T:
                continue
            lp = -G.ctc_loss_single(logits, list(lab), blank)[0]
            if best is None or lp > best[0]:
                best = (lp, list(lab))
    return best


@pytest.mark.parametrize("seed", range(6))
def test_beam_search_exhaustive_is_exact_argmax(seed):
    """With a beam wider than every prefix, prefix beam search is exact: the
    top path is the most probable labeling and its score is log p(labeling)."""
    rng = np.random.default_rng(seed)
    lg = rng.standard_normal((5, 3)) * 2
    lp, lab = _best_labeling(lg, 2)
    paths, lps = G.ctc_beam_search_single(lg, beam_width=64, merge_repeated=False)
    assert paths[0] == lab
    assert abs(lps[0] - lp) < 1e-9


def test_beam_search_labelseq_merge_quirk():
    """[TF1] LabelSeq(merge_repeated=True) also merges equal labels separated
    by a blank in the prefix (A B * B -> A B); merge_repeated=False keeps them."""
    hi, lo = 8.0, -8.0
    lg = np.full((4, 3), lo)
    lg[0, 0] = lg[1, 1] = lg[2, 2] = lg[3, 1] = hi          # A B blank B
    assert G.ctc_beam_search_single(lg, 8, merge_repeated=False)[0][0] == [0, 1, 1]
    assert G.ctc_beam_search_single(lg, 8, merge_repeated=True)[0][0] == [0, 1]
    assert G.ctc_greedy_decode(lg[:, None, :], np.array([4]), blank=2)[0] == [[0, 1, 1]]


def test_beam_search_top_paths_sorted_and_empty_sequence():
    rng = np.random.default_rng(3)
    lg = rng.standard_normal((6, 5))
    paths, lps = G.ctc_beam_search_single(lg, 10, top_paths=4)
    assert len(paths) == 4 and all(a >= b for a, b in zip(lps, lps[1:]))
    paths, lps = G.ctc_beam_search_single(lg[:0], 10)
    assert paths == [[]] and lps == [0.0]


def test_edit_distance_kat():
    assert G.edit_distance([1, 2, 3], [1, 2, 3]) == 0
    assert G.edit_distance([1, 3], [1, 2, 3]) == 1
    assert G.edit_distance([], [1, 2]) == 2
    assert G.edit_distance([4, 5, 6], [1, 2]) == 3
    cer, ser = G.label_and_sequence_error([[1, 3], [1]], [[1, 2, 3], [1]])
    assert cer == 1 / 4 and ser == 0.5


def test_adam_kat():
    p, m, v = G.adam_update(np.array([1.0]), np.array([0.5]), np.zeros(1), np.zeros(1), 0.1, 1)
    # first step: m = 0.05, v = 0.00025, lr_t = 0.1*sqrt(0.001)/0.1 -> p -= ~0.1
    np.testing.assert_allclose(p, 1.0 - 0.1 * np.sqrt(1e-3) / 0.1 * 0.05 / (np.sqrt(2.5e-4) + 1e-8))
    assert G.learning_rate(2 ** 16) == pytest.approx(0.9e-4)


# ------------------------------------------------------------ whole graph
@pytest.mark.parametrize("cell,sizes", [("gru", (512, 256)), ("lstm", (512, 512))])
def test_store_init_equals_oracle_init(cell, sizes):
    """ParamStore's reference initialisers walk variables in the reference's
    creation order, so a seed gives the oracle's values whatever the buffer layout."""
    from cnn_lstm_ctc_ocr_amd.config import ModelConfig
    from cnn_lstm_ctc_ocr_amd.params import reference_init
    a = reference_init(ModelConfig(cell=cell, rnn_sizes=sizes), seed=3)
    b = M.init_params(seed=3, cell=cell, rnn_sizes=sizes)
    assert set(a) == set(b)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_param_counts_match_survey():
    n = lambda shapes: sum(int(np.prod(s)) for k, s in shapes.items() if M.is_trainable(k))
    conv = sum(int(np.prod(s)) for k, s in M.param_shapes().items()
               if k.startswith("convnet") and k.split("/")[-1] in ("kernel", "bias"))
    assert conv == 1_171_680
    assert n(M.param_shapes("lstm", (512, 512))) == 10_716_416          # SURVEY a13 (incl. BN gamma/beta)
    assert n(M.param_shapes("gru", (512, 256))) == 5_551_872


@pytest.mark.parametrize("cell,sizes", [("lstm", (6, 5)), ("gru", (5, 4))])
def test_whole_graph_gradient_finite_difference(cell, sizes):
    """KAT for the composition: d(loss)/d(param) of the full graph (train mode,
    float64) against central differences on a handful of coordinates."""
    rng = np.random.default_rng(8)
    params = M.init_params(seed=3, cell=cell, rnn_sizes=sizes, dtype=np.float64)
    for k in params:                              # larger RNN weights: non-trivial grads
        if "cell" in k:
            params[k] = params[k] * 30
    B, W = 2, 36
    x = G.preprocess(rng.integers(0, 256, (B, 32, W, 1)).astype(np.uint8)).astype(np.float64)
    widths = np.array([36, 30])
    labels = [[1, 2], [3]]
    model = M.RefModel(params, cell, sizes)
    loss, grads, _, _, _ = model.loss_and_grads(x, widths, labels)

    def f(p):
        return M.RefModel(p, cell, sizes).loss_and_grads(x, widths, labels)[0]

    names = ["convnet/conv1/kernel", "convnet/conv4/batch_norm/gamma", "convnet/conv8/bias",
             "rnn/logits/kernel", "rnn/logits/bias"]
    names += [k for k in params if "bdrnn1/bw" in k][:1] + [k for k in params if "bdrnn2/fw" in k][:1]
    for name in names:
        flat = params[name].reshape(-1)
        for idx in rng.choice(flat.size, 2, replace=False):
            eps = 1e-6
            pp = {k: v.copy() for k, v in params.items()}
            pp[name].reshape(-1)[idx] += eps
            pm = {k: v.copy() for k, v in params.items()}
            pm[name].reshape(-1)[idx] -= eps
            fd = (f(pp) - f(pm)) / (2 * eps)
            an = grads[name].reshape(-1)[idx]
            assert abs(fd - an) <= 1e-5 * max(1.0, abs(fd)), (name, idx, fd, an)


def test_train_step_runs_and_updates():
    rng = np.random.default_rng(9)
    params = M.init_params(seed=1, rnn_sizes=(8, 8))
    x = G.preprocess(rng.integers(0, 256, (2, 32, 40, 1)).astype(np.uint8))
    loss, newp, state = M.train_step(params, {}, 0, x, np.array([40, 40]), [[1, 2, 3], [4]],
                                     rnn_sizes=(8, 8))
    assert np.isfinite(loss)
    assert not np.allclose(newp["rnn/logits/kernel"], params["rnn/logits/kernel"])
    assert not np.allclose(newp["convnet/conv2/batch_norm/moving_mean"], 0)


@pytest.mark.parametrize("cell", ["lstm", "gru"])
def test_torch_cpu_restatement_matches_oracle(cell):
    """oracle/torch_ref.py (the timed CPU baseline of bench.py) computes the
    oracle's graph: TRAIN-mode loss, logits-layer and conv1 gradients, and one
    TF1 Adam update, at a small full-width shape."""
    import torch

    from oracle.torch_ref import TorchRef
    rng = np.random.default_rng(9)
    sizes = (32, 32) if cell == "lstm" else (32, 16)
    vals = M.init_params(seed=3, cell=cell, rnn_sizes=sizes)
    for k in vals:
        if "_cell/" in k and "kernel" in k:
            vals[k] = (vals[k] * 20).astype(np.float32)
    B, W = 3, 64
    img = rng.integers(0, 256, (B, 32, W, 1)).astype(np.uint8)
    widths = np.full(B, W, np.int32)
    labels = [list(rng.integers(0, 95, n)) for n in (3, 5, 4)]
    ref = M.RefModel({k: v.astype(np.float64) for k, v in vals.items()}, cell, sizes)
    loss_ref, grads_ref, _, logits_ref, _ = ref.loss_and_grads(G.preprocess(img).astype(np.float64), widths, labels)
    tr = TorchRef(vals, sizes, dtype=torch.float64, cell=cell)
    lab = torch.zeros(B, 5, dtype=torch.long)
    for i, l in enumerate(labels):
        lab[i, :len(l)] = torch.tensor(l)
    ln = torch.tensor([len(l) for l in labels])
    logits = tr.forward(torch.from_numpy(img), True)
    np.testing.assert_allclose(logits.detach().numpy(), logits_ref, rtol=1e-9, atol=1e-9)
    loss = tr.loss(logits, lab, ln)
    loss.backward()
    assert abs(loss.item() - loss_ref) < 1e-9 * abs(loss_ref)
    rnn = "lstm_cell/kernel" if cell == "lstm" else "gru_cell/candidate/kernel"
    for name in ("rnn/logits/kernel", "rnn/bdrnn1/bw/" + rnn, "convnet/conv8/batch_norm/gamma",
                 "convnet/conv1/kernel"):
        np.testing.assert_allclose(tr.p[name].grad.numpy(), grads_ref[name], rtol=1e-7, atol=1e-10, err_msg=name)


@pytest.mark.parametrize("cell", ["lstm", "gru"])
def test_torch_cpu_restatement_masked_matches_oracle(cell):
    """The sequence_length-masked restatement (oracle/torch_ref.py: dynamic_rnn
    stop-and-carry, reverse_sequence for the backward direction,
    model_bu.py:187-192 / model.py:152-163) equals the NumPy oracle on a RAGGED
    batch: logits (including the zero-output padded steps), the per-row CTC loss
    over seq_len and gradients through both directions -- the float64 graph
    the fp32 C5 / ragged GPU tests compare against."""
    import torch

    from oracle.torch_ref import TorchRef
    rng = np.random.default_rng(11)
    sizes = (32, 32) if cell == "lstm" else (32, 16)
    vals = M.init_params(seed=4, cell=cell, rnn_sizes=sizes)
    for k in vals:
        if "_cell/" in k and "kernel" in k:
            vals[k] = (vals[k] * 20).astype(np.float32)
    B, W = 4, 96
    widths = np.array([96, 41, 70, 57], np.int32)                 # seq_len 45, 17, 32, 25
    img = np.zeros((B, 32, W, 1), np.uint8)
    for b, w in enumerate(widths):
        img[b, :, :w] = rng.integers(0, 256, (32, w, 1))
    labels = [list(rng.integers(0, 95, n)) for n in (6, 3, 5, 4)]
    ref = M.RefModel({k: v.astype(np.float64) for k, v in vals.items()}, cell, sizes)
    loss_ref, grads_ref, losses_ref, logits_ref, seq_ref = ref.loss_and_grads(
        G.preprocess(img).astype(np.float64), widths, labels)
    assert len(set(seq_ref.tolist())) == B
    tr = TorchRef(vals, sizes, dtype=torch.float64, cell=cell)
    lab = torch.zeros(B, 6, dtype=torch.long)
    for i, l in enumerate(labels):
        lab[i, :len(l)] = torch.tensor(l)
    ln = torch.tensor([len(l) for l in labels])
    logits = tr.forward(torch.from_numpy(img), True, widths=widths)
    assert tr.seq_len.tolist() == seq_ref.tolist()
    np.testing.assert_allclose(logits.detach().numpy(), logits_ref, rtol=1e-9, atol=1e-9)
    losses = tr.loss(logits, lab, ln, per_sequence=True)
    np.testing.assert_allclose(losses.detach().numpy(), losses_ref, rtol=1e-9)
    (losses.sum() / B).backward()
    rnn = "lstm_cell/kernel" if cell == "lstm" else "gru_cell/candidate/kernel"
    for name in ("rnn/logits/kernel", "rnn/bdrnn1/bw/" + rnn, "rnn/bdrnn2/fw/" + rnn, "convnet/conv8/batch_norm/gamma",
                 "convnet/conv1/kernel"):
        np.testing.assert_allclose(tr.p[name].grad.numpy(), grads_ref[name], rtol=1e-7, atol=1e-10, err_msg=name)
    # full widths through the masked route equal the unmasked fast path
    full = np.full(B, W, np.int32)
    a = tr.forward(torch.from_numpy(img), False, widths=full).detach().numpy()
    b = tr.forward(torch.from_numpy(img), False).detach().numpy()
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12)
