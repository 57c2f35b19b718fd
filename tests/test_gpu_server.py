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


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_replica_pool_on_gpu_matches_single_recognizer(cuda, dtype):
    """Two replica PROCESSES behind one LocalServer give the single in-process
    Recognizer's strings. One replica per GPU where the box has two (cuda:0,
    cuda:1: each worker makes its own GPU current before building);
    both on cuda:0 on a one-GPU box. bf16 (allow_bf16) runs the ping-pong GEMM
    engines, whose LDS limits are set per device."""
    from cnn_lstm_ctc_ocr_amd import ModelConfig
    from cnn_lstm_ctc_ocr_amd.server import LocalServer, Recognizer, ReplicaPool, gpu_recognizer
    sizes = SIZES if dtype == torch.float32 else (256, 256)
    cfg = ModelConfig(rnn_sizes=sizes, dtype=dtype)
    rng = np.random.default_rng(8)
    widths = [int(w) for w in rng.integers(40, 300, 24)]
    crops = [rng.integers(0, 256, (32, w), dtype=np.uint8) for w in widths]

    def serve(rec):
        srv = LocalServer(rec, bucket_size=4, bucket_max_time=0.0)
        cid, _, outq = srv.register()
        for i, c in enumerate(crops):
            srv.addImage(cid, i, 0.0, c)
        for k in range(12):
            srv.flush_buckets(now=1e9 + k)
        srv.collect(block=True)
        got = {}
        while not outq.empty():
            i, t = outq.get()
            got[i] = t
        return got

    from cnn_lstm_ctc_ocr_amd import ParamStore
    bf = dtype == torch.bfloat16
    single = serve(Recognizer(ParamStore(cfg, device=cuda, seed=4), allow_bf16=bf))
    devices = ["cuda:0", "cuda:1"] if torch.cuda.device_count() > 1 else ["cuda:0", "cuda:0"]
    with ReplicaPool(devices, gpu_recognizer(cfg, seed=4, allow_bf16=bf)) as pool:
        multi = serve(pool)
    assert sorted(single) == list(range(len(crops))) and multi == single


def test_recognizer_refuses_bf16_store_unless_allowed(cuda):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.server import Recognizer
    store = ParamStore(ModelConfig(rnn_sizes=SIZES, dtype=torch.bfloat16), device=cuda, seed=0)
    with pytest.raises(ValueError, match="allow_bf16"):
        Recognizer(store)
    Recognizer(store, allow_bf16=True)
