"""Build tests/golden/mjsynth_test_bucket.npz: real MJSynth crops from the
reference's data/test shard (one width bucket, (96, 128]) through the
reference input-pipeline semantics, plus the float64 oracle's outputs with the
reference initialisers (seed 0, LSTM 512/512, model_bu.py).

    python tools/make_golden.py        (needs /root/reference/data; run here, not on the GPU box)

Stored: the preprocessed float32 batch exactly as mjsynth.py would feed it
(first-row pad, 0.0 dynamic padding), the raw uint8 crops right-padded with 0
as the serving path would (server.py:29-34), widths, labels, texts, and the
oracle's INFER logits, TRAIN-mode per-crop CTC losses, greedy and beam-16
decodes for both inputs.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from cnn_lstm_ctc_ocr_amd import input_pipeline as P  # noqa: E402
from cnn_lstm_ctc_ocr_amd.tfrecord import read_word_records  # noqa: E402
from oracle import ref_graph as G  # noqa: E402
from oracle import ref_model as M  # noqa: E402

N, LO, HI = 8, 96, 128


def main():
    recs = []
    for r in read_word_records("/root/reference/data/test/words-000.tfrecord"):
        if LO < r["width"] <= HI:
            recs.append(r)
        if len(recs) == N:
            break
    crops = [P.decode_jpeg_gray(r["image"]) for r in recs]
    items = [{"image": P.preprocess_image(c), "width": r["width"], "labels": r["labels"], "length": r["length"],
              "text": r["text"], "filename": r["filename"]} for c, r in zip(crops, recs)]
    image, width, (idx, vals, shape), length, text, _ = P.make_batch(items)
    x_f32 = image.numpy()
    widths = width.numpy()
    labels = [list(map(int, r["labels"])) for r in recs]
    lab = np.zeros((N, max(len(l) for l in labels)), np.int32)
    for i, l in enumerate(labels):
        lab[i, :len(l)] = l
    lab_len = np.array([len(l) for l in labels], np.int32)
    # serving layout: uint8, 32 rows (first-row pad), right zero padding to the bucket width
    u8 = np.zeros((N, 32, HI, 1), np.uint8)
    for i, c in enumerate(crops):
        c = np.concatenate([c[:1], c], 0)[:32]
        u8[i, :c.shape[0], :c.shape[1]] = c

    vals0 = {k: v.astype(np.float64) for k, v in M.init_params(seed=0).items()}
    ref = M.RefModel(vals0, "lstm", (512, 512))
    out = {"x_f32": x_f32, "x_u8": u8, "widths": widths, "labels": lab, "label_len": lab_len,
           "texts": np.array(text)}
    for tag, x in (("f32", x_f32.astype(np.float64)), ("u8", G.preprocess(u8).astype(np.float64))):
        logits, seq = ref.forward(x, widths, training=False)
        out[f"{tag}_logits"] = logits.astype(np.float32)
        out[f"{tag}_seq_len"] = seq.astype(np.int32)
        out[f"{tag}_greedy"] = G.to_dense(G.ctc_greedy_decode(logits, seq)[0])
        paths, logp = G.ctc_beam_search_decode(logits, seq, beam_width=16)
        out[f"{tag}_beam16"] = G.to_dense(paths[0])
        out[f"{tag}_beam16_logp"] = logp[:, 0].astype(np.float32)
    loss, _, _, _, _ = ref.loss_and_grads(x_f32.astype(np.float64), widths, labels)
    out["f32_train_loss"] = np.float64(loss)
    path = os.path.join(ROOT, "tests", "golden", "mjsynth_test_bucket.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), "bytes;", {k: getattr(v, "shape", v) for k, v in out.items()})


if __name__ == "__main__":
    main()
