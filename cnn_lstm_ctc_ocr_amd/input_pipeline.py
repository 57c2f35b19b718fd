"""Drop-in for the training/eval input pipelines of src/weinman/mjsynth.py
(bucketed_input_pipeline :28-77, threaded_input_pipeline :79-113) without
TensorFlow: TFRecord shards -> JPEG decode -> preprocess -> filter ->
bucket_by_sequence_length -> dynamically padded batches on the device.

Semantics followed:
  * _read_word_record (:148-172): features image/encoded, image/labels,
    image/width, image/filename, text/string, text/length (tfrecord.py);
  * decode_jpeg(channels=1): libjpeg's grayscale output (PIL draft mode 'L'
    decodes straight to the Y channel, no RGB round trip). TF itself is not
    available here, so bit-parity of the decode is unpinned; every GPU parity
    test feeds uint8 arrays instead;
  * _preprocess_image (:185-194): float32(x) * float32(1/255) - 0.5, then the
    first row is duplicated (31 -> 32 rows) -- BEFORE batching, so the
    dynamic padding value 0.0 is mid-gray, unlike serving's uint8 0 (-0.5);
  * _get_input_filter (:115-144): keep width <= width_threshold and
    length <= length_threshold (either optional);
  * tf.contrib.training.bucket_by_sequence_length(width, boundaries): bucket i
    holds boundaries[i-1] <= width < boundaries[i] (len(boundaries)+1
    buckets); a bucket emits when it holds batch_size crops; with a finite
    num_epochs (allow_smaller_final_batch) the leftovers are emitted at the end;
  * string_input_producer(shuffle=True): a fresh file order per epoch (seeded
    here so runs are reproducible);
  * labels: SparseTensor int32 (indices [N,2] int64, values [N], dense_shape).
"""
import bisect
import glob
import io
import os

import numpy as np
import torch

from .tfrecord import read_word_records

DEFAULT_BOUNDARIES = (32, 64, 96, 128, 160, 192, 224, 256)      # mjsynth.py:31
_INV255 = np.float32(1.0 / 255.0)


def decode_jpeg_gray(data):
    """tf.image.decode_jpeg(contents, channels=1) -> uint8 [H, W, 1]."""
    from PIL import Image
    im = Image.open(io.BytesIO(data))
    if im.format == "JPEG":
        im.draft("L", im.size)
    if im.mode != "L":
        im = im.convert("L")
    return np.asarray(im, dtype=np.uint8)[:, :, None]


def preprocess_image(img_u8):
    """mjsynth._preprocess_image: uint8 [H, W, 1] -> float32 [H+1, W, 1]."""
    x = img_u8.astype(np.float32) * _INV255 - np.float32(0.5)
    return np.concatenate([x[:1], x], axis=0)


def keep_input(width, width_threshold, length, length_threshold):
    """mjsynth._get_input_filter."""
    keep = True
    if width_threshold is not None:
        keep = keep and width <= width_threshold
    if length_threshold is not None:
        keep = keep and length <= length_threshold
    return keep


def bucket_index(width, boundaries):
    """Bucket of bucket_by_sequence_length: #boundaries <= width."""
    return bisect.bisect_right(list(boundaries), width)


def data_files(base_dir, file_patterns):
    """mjsynth._get_data_queue's file list (glob per pattern, flattened)."""
    out = []
    for pat in file_patterns:
        out += sorted(glob.glob(os.path.join(base_dir, pat)))
    return out


def _examples(files, num_epochs, shuffle, seed):
    rng = np.random.default_rng(seed)
    epoch = 0
    while num_epochs is None or epoch < num_epochs:
        order = list(files)
        if shuffle:
            rng.shuffle(order)
        for f in order:
            for rec in read_word_records(f):
                yield rec
        epoch += 1
        if not files:
            return


def _sparse(labels):
    idx = [(b, t) for b, lab in enumerate(labels) for t in range(len(lab))]
    vals = [v for lab in labels for v in lab]
    lmax = max([len(lab) for lab in labels] + [0])
    return (np.asarray(idx, np.int64).reshape(-1, 2), np.asarray(vals, np.int32),
            np.asarray([len(labels), lmax], np.int64))


def make_batch(items, device=None, dtype=torch.float32):
    """dynamic_pad: every image zero-padded (0.0) at the bottom/right to the
    batch's max height and width -- MJSynth crops are 23..32 rows, so after
    the first-row pad a batch is usually 32 or 33 rows, which the conv tower
    reduces to one row all the same. Returns the reference tuple (image,
    width, label, length, text, filename)."""
    wmax = max(it["image"].shape[1] for it in items)
    hmax = max(it["image"].shape[0] for it in items)
    img = np.zeros((len(items), hmax, wmax, 1), np.float32)
    for i, it in enumerate(items):
        h, w = it["image"].shape[:2]
        img[i, :h, :w] = it["image"]
    image = torch.from_numpy(img)
    width = torch.tensor([it["width"] for it in items], dtype=torch.int32)
    length = torch.tensor([it["length"] for it in items], dtype=torch.int64)
    if device is not None:
        image = image.to(device=device, dtype=dtype, non_blocking=True)
        width = width.to(device, non_blocking=True)
        length = length.to(device, non_blocking=True)
    label = _sparse([it["labels"] for it in items])
    return image, width, label, length, [it["text"] for it in items], [it["filename"] for it in items]


def _decoded(recs, width_threshold, length_threshold):
    for r in recs:
        if not keep_input(r["width"], width_threshold, r["length"], length_threshold):
            continue
        img = decode_jpeg_gray(r["image"])
        yield {"image": preprocess_image(img), "width": r["width"], "labels": r["labels"],
               "length": r["length"], "text": r["text"], "filename": r["filename"]}


def bucketed_input_pipeline(base_dir, file_patterns, batch_size=32, boundaries=DEFAULT_BOUNDARIES,
                            width_threshold=None, length_threshold=None, num_epochs=None, device=None,
                            dtype=torch.float32, seed=0, shuffle_files=True):
    """Generator of (image [B,32,Wmax,1], width i32 [B], label sparse triple,
    length i64 [B], text list, filename list) bucketed by width."""
    files = data_files(base_dir, file_patterns)
    buckets = [[] for _ in range(len(boundaries) + 1)]
    for it in _decoded(_examples(files, num_epochs, shuffle_files, seed), width_threshold, length_threshold):
        q = buckets[bucket_index(it["width"], boundaries)]
        q.append(it)
        if len(q) == batch_size:
            yield make_batch(q, device, dtype)
            q.clear()
    if num_epochs is not None:                        # allow_smaller_final_batch
        for q in buckets:
            if q:
                yield make_batch(q, device, dtype)


def threaded_input_pipeline(base_dir, file_patterns, batch_size=32, num_epochs=None, device=None,
                            dtype=torch.float32, seed=0, shuffle_files=True):
    """batch_join with dynamic_pad, no bucketing (mjsynth.py:79-113)."""
    files = data_files(base_dir, file_patterns)
    q = []
    for it in _decoded(_examples(files, num_epochs, shuffle_files, seed), None, None):
        q.append(it)
        if len(q) == batch_size:
            yield make_batch(q, device, dtype)
            q = []
    if num_epochs is not None and q:
        yield make_batch(q, device, dtype)
