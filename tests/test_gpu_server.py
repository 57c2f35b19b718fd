"""The recognise service (server.py / linepredictor.py drop-ins) with the GPU
recogniser against the oracle run on the same bucketed, padded batch."""
import threading

import numpy as np
import pytest
import torch

from oracle import ref_graph as G
from oracle import ref_model as M

pytestmark = pytest.mark.gpu
SIZES = (64, 64)


def _store(cuda, seed=0):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    vals = M.init_params(seed=seed, rnn_sizes=SIZES)
    for k in vals:
        if "lstm_cell/kernel" in k:
            vals[k] = (vals[k] * 20).astype(np.float32)
    return ParamStore(ModelConfig(rnn_sizes=SIZES, dtype=torch.float32), device=cuda, values=vals), vals


@pytest.mark.parametrize("decoder", ["greedy", "beam"])
def test_recognizer_matches_oracle_on_bucket_batch(cuda, decoder):
    from cnn_lstm_ctc_ocr_amd.mjsynth import out_charset
    from cnn_lstm_ctc_ocr_amd.server import Bucket, Recognizer, fill_batch
    store, vals = _store(cuda)
    rng = np.random.default_rng(1)
    b = Bucket(0.0, 16, (96, 128))
    widths = rng.integers(97, 129, 13)
    for i, w in enumerate(widths):
        b.addImgToBucket("0", str(i), 0.0, rng.integers(0, 256, (32, int(w))).astype(np.uint8))
    infos, batch, wd = fill_batch(*b.getBatch(now=1.0), 16)
    rec = Recognizer(store, decoder=decoder, beam_width=16)
    texts = rec(batch, wd)
    logits_ref, seq_ref = M.RefModel(vals, "lstm", SIZES).forward(G.preprocess(batch), wd, training=False)
    if decoder == "greedy":
        seqs, _ = G.ctc_greedy_decode(logits_ref, seq_ref)
    else:
        seqs = G.ctc_beam_search_decode(logits_ref, seq_ref, beam_width=16)[0][0]
    want = ["".join(out_charset[c] for c in s) for s in seqs]
    assert texts == want


def test_service_end_to_end_on_gpu(cuda):
    from cnn_lstm_ctc_ocr_amd.linepredictor import BatchLinePredictor
    from cnn_lstm_ctc_ocr_amd.server import LocalServer, Recognizer
    store, vals = _store(cuda, seed=2)
    rec = Recognizer(store)
    srv = LocalServer(rec, bucket_size=8, bucket_max_time=0.0)
    client = BatchLinePredictor(srv)
    rng = np.random.default_rng(3)
    crops = [rng.integers(0, 256, (32, int(w))).astype(np.uint8) for w in rng.integers(40, 300, 20)]
    stop = threading.Event()
    th = threading.Thread(target=srv.run, kwargs={"stop": stop.is_set, "idle_sleep": 0.001})
    th.start()
    try:
        got = client.predict_batch("page", crops, give_up_after=50000)
    finally:
        stop.set()
        th.join()
    # each crop alone, padded to its bucket, must read the same (row independence)
    for i, c in enumerate(crops):
        w = c.shape[1]
        bw = -(-w // 32) * 32
        x = np.zeros((1, 32, bw, 1), np.uint8)
        x[0, :, :w, 0] = c
        assert rec(x, np.array([w], np.int32))[0] == got[i], i
