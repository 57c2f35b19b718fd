"""Build tests/golden/mjsynth_{val,test}_words000.npz: every crop of the
reference's data/val/words-000.tfrecord (803 MJSynth word crops: the training
shard of tests/test_gpu_trained.py) and data/test/words-000.tfrecord (the
held-out shard: trained-weight decode parity and held-out CER) as DATA --
decoded uint8 pixels, widths, labels and texts. No reference source is stored;
the GPU box has no /root/reference, so this is how the shards travel.

    python tools/make_val_fixture.py [val|test]    (needs /root/reference/data; run here)

Decode: input_pipeline.decode_jpeg_gray (libjpeg grayscale via PIL; TF's
decode_jpeg is unavailable, so bit-parity of the JPEG decode is unpinned --
the test consumes these uint8 arrays, not JPEGs). Crops are 23..32 rows
(heights[i]); the pixels are stored side by side, [32, sum(widths)], crop i in
rows 0 .. heights[i] and columns offsets[i] .. offsets[i] + widths[i] (rows
below its height are 0 and not part of it). Labels are checked against the text
(mjsynth.out_charset), as tests/test_oracle.py does for the whole shard.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from cnn_lstm_ctc_ocr_amd import input_pipeline as P  # noqa: E402
from cnn_lstm_ctc_ocr_amd.tfrecord import read_word_records  # noqa: E402
from oracle import ref_graph as G  # noqa: E402

SRC = "/root/reference/data/{}/words-000.tfrecord"


def main(split="val"):
    recs = list(read_word_records(SRC.format(split)))
    crops = [P.decode_jpeg_gray(r["image"])[:, :, 0] for r in recs]
    heights = np.array([c.shape[0] for c in crops], np.int32)
    assert heights.max() <= 32
    widths = np.array([c.shape[1] for c in crops], np.int32)
    assert widths.tolist() == [int(r["width"]) for r in recs]
    offsets = np.concatenate([[0], np.cumsum(widths)[:-1]]).astype(np.int64)
    pixels = np.zeros((32, int(widths.sum())), np.uint8)
    for c, o in zip(crops, offsets):
        pixels[:c.shape[0], o:o + c.shape[1]] = c
    lmax = max(int(r["length"]) for r in recs)
    labels = np.zeros((len(recs), lmax), np.int32)
    for i, r in enumerate(recs):
        lab = [int(v) for v in r["labels"]]
        assert lab == G.encode_text(r["text"])
        labels[i, :len(lab)] = lab
    out = {"pixels": pixels, "offsets": offsets, "widths": widths, "heights": heights, "labels": labels,
           "label_len": np.array([int(r["length"]) for r in recs], np.int32),
           "texts": np.array([r["text"] for r in recs])}
    path = os.path.join(ROOT, "tests", "golden", f"mjsynth_{split}_words000.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), "bytes;", {k: getattr(v, "shape", v) for k, v in out.items()})


if __name__ == "__main__":
    main(*sys.argv[1:2])
