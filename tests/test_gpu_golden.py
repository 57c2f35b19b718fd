"""Real MJSynth crops (tests/golden/mjsynth_test_bucket.npz, made by
tools/make_golden.py from the reference's data/test shard) through the GPU
path with the reference initialisers (seed 0, LSTM 512/512, fp32), against the
float64 oracle's stored outputs."""
import os

import numpy as np
import pytest
import torch

from oracle import ref_graph as G

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(__file__), "golden", "mjsynth_test_bucket.npz")


@pytest.fixture(scope="module")
def golden():
    with np.load(FIX, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def store(cuda):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    return ParamStore(ModelConfig(dtype=torch.float32), device=cuda, seed=0)


def _no_near_tie(logits, seq, b, rel=1e-4):
    top2 = np.sort(logits[:seq[b], b], axis=1)[:, -2:]
    return np.all(top2[:, 1] - top2[:, 0] > rel * max(1.0, np.abs(logits).max()))


@pytest.mark.parametrize("tag", ["f32", "u8"])
def test_golden_infer_logits_and_decodes(cuda, golden, store, tag):
    from cnn_lstm_ctc_ocr_amd import decode, model
    x = torch.from_numpy(golden[f"x_{tag}"]).to(cuda)
    widths = torch.from_numpy(golden["widths"]).to(cuda)
    with torch.no_grad():
        feats, seq = model.convnet_layers(x, widths, model.INFER, store)
        logits = model.rnn_layers(feats, seq, 95, store)
        greedy = decode.ctc_greedy_decoder(logits, seq)[0][0].cpu().numpy()
        beam, logp = decode.ctc_beam_search_decoder(logits, seq, beam_width=16)
    lg = logits.cpu().numpy()
    want = golden[f"{tag}_logits"]
    assert seq.cpu().numpy().tolist() == golden[f"{tag}_seq_len"].tolist()
    assert np.linalg.norm(lg - want) / np.linalg.norm(want) < 1e-4
    g_want = golden[f"{tag}_greedy"]
    for b in range(lg.shape[1]):
        if _no_near_tie(want, golden[f"{tag}_seq_len"], b):
            row = greedy[b][greedy[b] >= 0].tolist() if greedy.shape[1] else []
            assert row == g_want[b][g_want[b] >= 0].tolist(), b
    # beam: bit-exact on the device's own logits, log-probs close to the oracle's
    paths_dev, _ = G.ctc_beam_search_decode(lg, seq.cpu().numpy(), beam_width=16)
    got = beam[0].cpu().numpy()
    assert [got[b][got[b] >= 0].tolist() for b in range(got.shape[0])] == paths_dev[0]
    np.testing.assert_allclose(logp[:, 0].cpu().numpy(), golden[f"{tag}_beam16_logp"], rtol=1e-4, atol=1e-3)


def test_golden_train_mode_loss(cuda, golden, store):
    from cnn_lstm_ctc_ocr_amd import model
    from cnn_lstm_ctc_ocr_amd.params import reference_init
    store.load_state_dict(reference_init(store.cfg, seed=0))       # BN moving stats untouched by other tests
    x = torch.from_numpy(golden["x_f32"]).to(cuda)
    widths = torch.from_numpy(golden["widths"]).to(cuda)
    lab = (torch.from_numpy(golden["labels"]).to(cuda), torch.from_numpy(golden["label_len"]).to(cuda))
    with torch.no_grad():
        feats, seq = model.convnet_layers(x, widths, model.TRAIN, store)
        loss = model.ctc_loss_layer(model.rnn_layers(feats, seq, 95, store), lab, seq)
    assert abs(loss.item() - float(golden["f32_train_loss"])) / float(golden["f32_train_loss"]) < 1e-4
