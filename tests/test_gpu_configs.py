"""BASELINE.json configurations as parity cases:
C2 -- B=64 synthetic 32x256 crops, forward + CTC loss + greedy decode, fp32,
      LSTM 512/512 with the reference initialisers;
C5 -- variable-width 32x{64..512} bucketed batches, beam-16 decode;
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
    # INFER rows are independent: the float64 oracle checks 8 of the 64 rows
    n = 8
    vals = {k: v.astype(np.float64) for k, v in M.init_params(seed=0).items()}
    logits_ref, seq_ref = M.RefModel(vals, "lstm", (512, 512)).forward(
        G.preprocess(img[:n]).astype(np.float64), widths[:n], training=False)
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


def test_c5_variable_width_buckets_beam16(cuda):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.server import Bucket, Recognizer, fill_batch
    store = ParamStore(ModelConfig(dtype=torch.bfloat16), device=cuda, seed=0)
    rec = Recognizer(store, decoder="beam", beam_width=16)
    rng = np.random.default_rng(5)
    for lo in (64, 224, 480):
        b = Bucket(0.0, 32, (lo, lo + 32))
        for i, w in enumerate(rng.integers(lo + 1, lo + 33, 27)):
            b.addImgToBucket("0", str(i), 0.0, rng.integers(0, 256, (32, int(w))).astype(np.uint8))
        infos, batch, widths = fill_batch(*b.getBatch(now=1.0), 32)
        with torch.no_grad():
            from cnn_lstm_ctc_ocr_amd import decode, model
            feats, seq = model.convnet_layers(torch.from_numpy(batch).to(cuda), torch.from_numpy(widths),
                                              model.INFER, store)
            logits = model.rnn_layers(feats, seq, 95, store).float()
            out, logp = decode.ctc_beam_search_decoder(logits, seq, beam_width=16)
        lg, sl = logits.cpu().numpy(), seq.cpu().numpy()
        sub = slice(0, 6)                                            # oracle beam search is slow in Python
        paths, lp = G.ctc_beam_search_decode(lg[:, sub], sl[sub], beam_width=16)
        got = out[0].cpu().numpy()[sub]
        assert [g[g >= 0].tolist() for g in got] == paths[0], lo
        np.testing.assert_allclose(logp.cpu().numpy()[sub, 0], lp[:, 0], rtol=1e-4, atol=2e-3)
        texts = rec(batch, widths)
        assert len(texts) == 32


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
