"""BASELINE.json configurations as parity cases:
C2 -- B=64 synthetic 32x256 crops, forward + CTC loss + greedy decode, fp32,
      LSTM 512/512 with the reference initialisers;
C5 -- variable-width 32x{64..512} bucketed batches, beam-16 decode, fp32 (the
      exact bench.py --config c5 workload, against the masked float64 graph);
plus the TF-Serving top-3 signature of client.py."""
import numpy as np
import pytest
import torch

from oracle import ref_graph as G
from oracle import ref_model as M

pytestmark = pytest.mark.gpu


def _labels(rng, B, T):
    out = []
    for _ in range(B):
        while True:
            L = int(rng.integers(2, 20))
            s = list(rng.integers(0, 95, L))
            if G.ctc_required_time(s) <= T:
                break
        out.append(s)
    return out


def test_c2_forward_ctc_greedy_fp32(cuda):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, kernels as K, model, validate
    store = ParamStore(ModelConfig(dtype=torch.float32), device=cuda, seed=0)
    rng = np.random.default_rng(20260)
    B, W = 64, 256
    img = rng.integers(0, 256, (B, 32, W, 1)).astype(np.uint8)
    widths = np.full(B, W, np.int32)
    T = G.seq_len_from_width([W])[0]
    labels = _labels(rng, B, T)
    with torch.no_grad():
        feats, seq = model.convnet_layers(torch.from_numpy(img).to(cuda), torch.from_numpy(widths), model.INFER, store)
        logits = model.rnn_layers(feats, seq, 95, store)
        lab, ln = model.dense_labels(labels, B, cuda)
        loss_b, _, status = K.ctc_loss(logits.contiguous(), lab, ln, seq, need_grad=False)
        dense = validate._get_output(logits, seq)[0].cpu().numpy()
    assert (status.cpu().numpy() == 0).all()
    # every row (8 of 64 were checked) against the reference graph in
    # float64 (oracle/torch_ref.py, pinned to the NumPy oracle in test_oracle.py;
    # full-width crops, so its unmasked recurrence is exact here)
    from oracle.torch_ref import TorchRef
    n = B
    vals = {k: v.astype(np.float64) for k, v in M.init_params(seed=0).items()}
    with torch.no_grad():
        logits_ref = TorchRef(vals, (512, 512), torch.float64).forward(torch.from_numpy(img), training=False).numpy()
    seq_ref = np.full(B, T, np.int64)
    lg = logits.cpu().numpy()
    assert np.linalg.norm(lg[:, :n] - logits_ref) / np.linalg.norm(logits_ref) < 1e-4
    loss_ref = [G.ctc_loss_single(logits_ref[:, b], labels[b], 95)[0] for b in range(n)]
    np.testing.assert_allclose(loss_b.cpu().numpy()[:n], loss_ref, rtol=1e-3)      # north_star: 1e-3 rel
    seqs, _ = G.ctc_greedy_decode(lg, seq.cpu().numpy())
    assert G.to_dense(seqs).tolist() == dense.tolist()              # decoder bit-exact on device logits
    seqs_ref, _ = G.ctc_greedy_decode(logits_ref, seq_ref)
    top2 = np.sort(logits_ref, axis=2)[:, :, -2:]
    for b in range(n):
        if np.all(top2[:seq_ref[b], b, 1] - top2[:seq_ref[b], b, 0] > 1e-4 * np.abs(logits_ref).max()):
            assert seqs[b] == seqs_ref[b], b


def _beam_rows(args):
    lg, sl = args
    paths, lp = G.ctc_beam_search_decode(lg, sl, beam_width=16, top_paths=2)
    return paths[0][0], lp[0]


def _pick(widths, n):
    """n rows of a bucket spread over its width range (shortest and longest included)."""
    order = np.argsort(widths, kind="stable")
    return np.unique(order[np.linspace(0, len(order) - 1, n).round().astype(int)])


def test_c5_fp32_buckets_vs_masked_float64_graph(cuda):
    """The route `bench.py --config c5` times, on its own workload: all 14
    width buckets of bench.c5_buckets (2,048 crops, true widths 65..512, each
    bucket a full batch of 107-160 crops zero-padded to its upper width, T up to
    253), fp32 store (the serving precision, server.Recognizer's default),
    convnet_layers -> rnn_layers -> beam-16 decode. Per bucket, 16 rows spread
    over its width range (rows are independent in INFER mode) against the
    reference graph in float64 with sequence_length masking
    (oracle/torch_ref.py, pinned to the NumPy oracle on ragged batches in
    test_oracle.py): seq_len exact, logits <= 1e-4 relative L2 (every step,
    padded steps included: they are relu(bias) in both), beam-16 paths bit-exact
    against the literal TF1 restatement on the device's logits, and against it
    on the float64 logits wherever the restatement's top-2 beam gap is not a
    near-tie."""
    import multiprocessing as mp
    import sys

    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, decode, model
    from oracle.torch_ref import TorchRef
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
    import bench
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=torch.float32), device=cuda, seed=0)
    ref = TorchRef({k: v.astype(np.float64) for k, v in M.init_params(seed=0).items()}, (512, 512), torch.float64)
    buckets = bench.c5_buckets()
    assert len(buckets) == 14 and max(u for u, _, _ in buckets) == 512
    cases = []
    for u, img, w in buckets:
        with torch.no_grad():
            feats, seq = model.convnet_layers(torch.from_numpy(img).to(cuda), torch.from_numpy(w), model.INFER, store)
            logits = model.rnn_layers(feats, seq, 95, store)
            out, logp = decode.ctc_beam_search_decoder(logits, seq, beam_width=16)
        seq = seq.cpu().numpy()
        assert seq.tolist() == G.seq_len_from_width(w).tolist(), u
        rows = _pick(w, 16)
        lg = logits.cpu().numpy()[:, rows]
        with torch.no_grad():
            lr = ref.forward(torch.from_numpy(img[rows]), training=False, widths=w[rows]).numpy()
        err = np.linalg.norm(lg - lr) / np.linalg.norm(lr)
        assert err < 1e-4, (u, err)
        for j in range(len(rows)):
            e = np.linalg.norm(lg[:, j] - lr[:, j]) / np.linalg.norm(lr[:, j])
            assert e < 3e-4, (u, rows[j], e)
        got = out[0].cpu().numpy()[rows]
        cases.append((u, rows, lg, lr, seq[rows], got, logp.cpu().numpy()[rows, 0]))
    jobs = []
    for _u, rows, lg, lr, sl, _g, _l in cases:
        for j in range(len(rows)):
            jobs.append((lg[:, j:j + 1], sl[j:j + 1]))
            jobs.append((lr[:, j:j + 1], sl[j:j + 1]))
    with mp.get_context("spawn").Pool(min(16, len(jobs))) as pool:
        res = pool.map(_beam_rows, jobs, chunksize=2)
    k, ties, checked = 0, 0, 0
    for u, rows, _lg, _lr, _sl, got, lp in cases:
        for j in range(len(rows)):
            (p_dev, lp_dev), (p_ref, lp_ref) = res[k], res[k + 1]
            k += 2
            path = got[j][got[j] >= 0].tolist()
            assert path == p_dev, (u, rows[j])                       # decoder bit-exact on the device logits
            np.testing.assert_allclose(lp[j], lp_dev[0], rtol=1e-4, atol=2e-3, err_msg=f"{u} {rows[j]}")
            if lp_ref[0] - lp_ref[1] > 1e-3:                          # end to end, off near-ties
                assert path == p_ref, (u, rows[j])
                checked += 1
            else:
                ties += 1
    assert checked >= 0.75 * (checked + ties), (checked, ties)          # measured 196 of 224


def test_serving_signature_top3(cuda):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.server import predict_signature
    store = ParamStore(ModelConfig(rnn_sizes=(64, 64), dtype=torch.float32), device=cuda, seed=3)
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (4, 32, 96, 1)).astype(np.uint8)
    sig = predict_signature(store, imgs, [96] * 4, beam_width=32)
    assert sorted(sig) == ["output0", "output1", "output2", "output3"]
    assert sig["output0"].shape == (4, 3)
    assert np.all(np.diff(sig["output0"], axis=1) <= 0)          # paths in descending probability
