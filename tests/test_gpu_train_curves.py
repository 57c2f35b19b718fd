"""Does the benched bf16 train step train like the reference's fp32 one?
(VERDICT r3 next #7.) The reference trains in fp32 (model_bu.py:187-192,
train.py:168-201); bench.py's headline step computes in bf16. Here both
precisions train the LSTM 512/512 model from the same seed on the reference's
own data -- every crop of data/val/words-000.tfrecord (tests/golden/
mjsynth_val_words000.npz, tools/make_val_fixture.py) through the training input
semantics (first-row pad, 0.0 dynamic padding, mjsynth.py:185-194) in width-
sorted batches of 32 -- for STEPS Trainer.step calls with the reference's
optimiser (Adam, lr 1e-4 exponential decay, train.py:120-137), and then decode
the shard with each trained model (greedy, validate.py:81-92) and score it
(CER = total edit distance / total label length, test.py:90-99).

Tolerances (stated, measured on MI355X; the curves are written to
$OCRK_CURVES_OUT when set): every 25-step window's mean loss of the bf16 run
within 5 % of the fp32 run's, both curves falling, and the shard CERs within
0.05 of each other."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
STEPS = 300
WINDOW = 25
FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "mjsynth_val_words000.npz")


def _batches(device):
    from cnn_lstm_ctc_ocr_amd import input_pipeline as P
    g = np.load(FIXTURE)
    order = np.argsort(g["widths"], kind="stable")
    items = []
    for i in order:
        o, w, h = int(g["offsets"][i]), int(g["widths"][i]), int(g["heights"][i])
        crop = g["pixels"][:h, o:o + w, None]
        n = int(g["label_len"][i])
        items.append({"image": P.preprocess_image(crop), "width": w, "labels": g["labels"][i, :n].tolist(),
                      "length": n, "text": str(g["texts"][i]), "filename": str(i)})
    out = []
    for k in range(len(items) // 32):
        image, width, _label, _len, _text, _fn = P.make_batch(items[32 * k:32 * k + 32])
        labels = [it["labels"] for it in items[32 * k:32 * k + 32]]
        out.append((image, width, labels))
    return out


def _train_and_score(dtype, batches, device):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, decode, model
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=dtype), device=device, seed=0)
    tr = Trainer(store)
    rng = np.random.default_rng(7)
    dev_batches = [(img.to(device=device, dtype=dtype), w, lab) for img, w, lab in batches]
    losses = []
    order = []
    while len(order) < STEPS:
        order += list(rng.permutation(len(dev_batches)))
    for i in order[:STEPS]:
        img, w, lab = dev_batches[i]
        losses.append(tr.step(img, w, lab))
    tr.check_status()
    losses = [float(v) for v in torch.stack(losses).cpu()]
    edits, total = 0.0, 0
    with torch.no_grad():
        for img, w, lab in dev_batches:
            feats, seq = model.convnet_layers(img, w, model.INFER, store)
            logits = model.rnn_layers(feats, seq, 95, store).float()
            hyp = decode.ctc_greedy_decoder(logits, seq)[0][0]
            ref, ref_len = model.dense_labels(lab, len(lab), device)
            hyp_len = (hyp >= 0).sum(1).to(torch.int32)
            d = decode.edit_distance(hyp, hyp_len, ref, ref_len)
            edits += float(d.sum())
            total += int(ref_len.sum())
    return np.array(losses), edits / total


def test_bf16_trains_like_fp32_on_reference_shard(cuda):
    batches = _batches(cuda)
    assert len(batches) == 25
    l32, cer32 = _train_and_score(torch.float32, batches, cuda)
    l16, cer16 = _train_and_score(torch.bfloat16, batches, cuda)
    w32 = l32.reshape(-1, WINDOW).mean(1)
    w16 = l16.reshape(-1, WINDOW).mean(1)
    rel = np.abs(w16 - w32) / w32
    if os.environ.get("OCRK_CURVES_OUT"):
        with open(os.environ["OCRK_CURVES_OUT"], "w") as fh:
            json.dump({"steps": STEPS, "window": WINDOW, "fp32_loss": l32.tolist(), "bf16_loss": l16.tolist(),
                       "fp32_window_mean": w32.tolist(), "bf16_window_mean": w16.tolist(),
                       "window_rel_diff": rel.tolist(), "cer_fp32": cer32, "cer_bf16": cer16}, fh)
    print(f"windows fp32 {np.round(w32, 3).tolist()}\nwindows bf16 {np.round(w16, 3).tolist()}\n"
          f"max rel {rel.max():.4f}; CER fp32 {cer32:.4f} bf16 {cer16:.4f}")
    assert np.isfinite(l32).all() and np.isfinite(l16).all()
    assert w32[-1] < 0.5 * w32[0] and w16[-1] < 0.5 * w16[0]
    assert rel.max() < 0.05, rel
    assert abs(cer16 - cer32) < 0.05, (cer32, cer16)
