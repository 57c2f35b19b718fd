"""TFRecord + JPEG input pipeline (src/weinman/mjsynth.py drop-in) on CPU."""
import os

import numpy as np
import pytest

from cnn_lstm_ctc_ocr_amd import input_pipeline as P
from cnn_lstm_ctc_ocr_amd.mjsynth import encode
from cnn_lstm_ctc_ocr_amd.tfrecord import read_word_records

from conftest import REFERENCE_DATA

needs_data = pytest.mark.skipif(not os.path.isdir(REFERENCE_DATA), reason="reference data shards absent")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "mjsynth_test_bucket.npz")


def test_bucket_index_matches_bucket_by_sequence_length():
    b = (32, 64, 96)
    assert [P.bucket_index(w, b) for w in (1, 31, 32, 63, 64, 95, 96, 500)] == [0, 0, 1, 1, 2, 2, 3, 3]


def test_filter_thresholds_inclusive():
    assert P.keep_input(100, 100, 5, 5) and not P.keep_input(101, 100, 5, 5)
    assert not P.keep_input(10, None, 6, 5) and P.keep_input(10 ** 6, None, None, None)


def test_preprocess_first_row_and_scale():
    img = np.arange(6, dtype=np.uint8).reshape(2, 3, 1) * 50
    x = P.preprocess_image(img)
    assert x.shape == (3, 3, 1) and x.dtype == np.float32
    np.testing.assert_array_equal(x[0], x[1])
    np.testing.assert_array_equal(x[1:], img.astype(np.float32) * np.float32(1 / 255) - np.float32(0.5))


def test_make_batch_pads_height_and_width_with_zero():
    a = {"image": np.ones((32, 5, 1), np.float32), "width": 5, "labels": [1, 2], "length": 2, "text": "BC",
         "filename": "a"}
    b = {"image": np.ones((33, 7, 1), np.float32), "width": 7, "labels": [3], "length": 1, "text": "D",
         "filename": "b"}
    image, width, (idx, vals, shape), length, text, fn = P.make_batch([a, b])
    assert tuple(image.shape) == (2, 33, 7, 1)
    assert float(image[0, 32].sum()) == 0 and float(image[0, :, 5:].sum()) == 0
    assert idx.tolist() == [[0, 0], [0, 1], [1, 0]] and vals.tolist() == [1, 2, 3] and shape.tolist() == [2, 2]


@needs_data
def test_records_labels_are_the_charset_encoding_of_the_text():
    n = 0
    for r in read_word_records(os.path.join(REFERENCE_DATA, "test", "words-000.tfrecord"), verify_crc=True):
        assert r["labels"] == encode(r["text"]) and r["length"] == len(r["text"])
        n += 1
    assert n == 892


@needs_data
def test_bucketed_pipeline_one_epoch_covers_every_kept_record():
    base = os.path.join(REFERENCE_DATA, "test")
    kept = [r for r in read_word_records(os.path.join(base, "words-000.tfrecord"))
            if r["width"] <= 200 and r["length"] <= 12]
    seen = []
    for image, width, label, length, text, fn in P.bucketed_input_pipeline(
            base, ["*.tfrecord"], batch_size=16, width_threshold=200, length_threshold=12, num_epochs=1):
        ids = {P.bucket_index(int(w), P.DEFAULT_BOUNDARIES) for w in width}
        assert len(ids) == 1
        assert image.shape[2] == int(width.max()) and image.shape[1] in (32, 33)
        assert (length.numpy() <= 12).all()
        seen += fn
    assert sorted(seen) == sorted(r["filename"] for r in kept)


@needs_data
def test_golden_fixture_is_the_pipeline_batch():
    """tests/golden/mjsynth_test_bucket.npz holds exactly what the pipeline makes."""
    with np.load(GOLDEN, allow_pickle=False) as z:
        x, widths, texts = z["x_f32"], z["widths"], z["texts"]
    recs = [r for r in read_word_records(os.path.join(REFERENCE_DATA, "test", "words-000.tfrecord"))
            if 96 < r["width"] <= 128][:len(widths)]
    items = [{"image": P.preprocess_image(P.decode_jpeg_gray(r["image"])), "width": r["width"],
              "labels": r["labels"], "length": r["length"], "text": r["text"], "filename": r["filename"]}
             for r in recs]
    image, width, _, _, text, _ = P.make_batch(items)
    np.testing.assert_array_equal(image.numpy(), x)
    assert width.tolist() == widths.tolist() and text == texts.tolist()
