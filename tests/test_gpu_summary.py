"""JSONL summaries from the GPU train step and eval harness (SURVEY 5;
train.py:139, test.py:100-102): values equal the step's own device results."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_train_and_eval_summaries(cuda, tmp_path):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, model, summary
    from cnn_lstm_ctc_ocr_amd import test as evaluation
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(64, 64), dtype=torch.float32), device=cuda, seed=3)
    path = tmp_path / "train.jsonl"
    w = summary.SummaryWriter(str(path))
    tr = Trainer(store, summary=w, summary_every=2)
    rng = np.random.default_rng(0)
    B, W = 32, 128
    img = torch.from_numpy(rng.integers(0, 256, (B, 32, W, 1), dtype=np.uint8)).to(cuda)
    labels = [list(rng.integers(0, 95, 5)) for _ in range(B)]
    losses = [float(tr.step(img, np.full(B, W, np.int32), labels)) for _ in range(4)]
    with torch.no_grad():
        feats, seq = model.convnet_layers(img, torch.full((B,), W, dtype=torch.int32), model.INFER, store)
        logits = model.rnn_layers(feats, seq, 95, store)
        lab, ln = model.dense_labels(labels, B, cuda)
        loss, cer, seqerr = evaluation._get_testing(logits, seq, (lab, ln), beam_width=16, summary=w, step=4)
    w.close()
    recs = summary.read(str(path))
    assert [r["step"] for r in recs[:2]] == [2, 4]
    assert recs[0]["loss"] == pytest.approx(losses[1], rel=1e-6)
    assert recs[1]["loss"] == pytest.approx(losses[3], rel=1e-6)
    assert recs[1]["crops_per_sec"] > 0 and recs[0]["learning_rate"] == pytest.approx(1e-4 * 0.9 ** (1 / 65536))
    ev = recs[2]
    assert ev["step"] == 4 and ev["label_error"] == pytest.approx(float(cer)) and \
        ev["sequence_error"] == pytest.approx(float(seqerr)) and ev["loss"] == pytest.approx(float(loss))
