"""Width-bucketed recognise service (src/processing/server.py, linepredictor.py):
bucket semantics on CPU with a stand-in recogniser; the GPU recogniser in
tests/test_gpu_server.py."""
import threading

import numpy as np
import pytest

from cnn_lstm_ctc_ocr_amd.linepredictor import BatchLinePredictor
from cnn_lstm_ctc_ocr_amd.server import Bucket, LocalServer, fill_batch


def _crop(w, v=7):
    return np.full((32, w), v, np.uint8)


def test_bucket_ranges_and_right_zero_padding():
    b = Bucket(1.0, 4, (64, 96))
    assert not b.addImgToBucket("0", "a", 0.0, _crop(64))        # (64, 96] excludes 64
    assert b.addImgToBucket("0", "a", 0.0, _crop(65))
    assert b.addImgToBucket("0", "b", 0.0, _crop(96))
    assert not b.addImgToBucket("0", "c", 0.0, _crop(97))
    img = b.imgs[0]
    assert img.shape == (32, 96, 1) and img.dtype == np.uint8
    assert (img[:, :65] == 7).all() and (img[:, 65:] == 0).all()
    assert b.widths == [65, 96]


def test_bucket_releases_only_above_batchsize_or_after_maxtime():
    b = Bucket(1.0, 2, (32, 64))
    for i in range(2):
        b.addImgToBucket("0", str(i), 10.0, _crop(40))
    assert b.getBatch(now=10.5) is None               # exactly batchsize: waits (server.py:45 uses '>')
    b.addImgToBucket("0", "2", 10.2, _crop(50))
    infos, batch, widths = b.getBatch(now=10.5)
    assert [i for _, i in infos] == ["0", "1"] and batch.shape == (2, 32, 64, 1)
    assert widths.tolist() == [40, 40] and len(b.imgs) == 1
    assert b.getBatch(now=11.0) is None               # oldest reset to the release time
    assert b.getBatch(now=11.6) is not None           # maxtime elapsed


def test_fill_batch_uses_first_width_and_marks_fillers():
    infos, batch, widths = fill_batch([("0", "a")], np.ones((1, 32, 64, 1), np.uint8), np.array([50], np.int32), 3)
    assert infos == [("0", "a"), ("-1", "0"), ("-1", "0")]
    assert widths.tolist() == [50, 50, 50] and (batch[1:] == 0).all()


def test_width_32_fits_no_bucket_unless_fixed():
    srv = LocalServer(lambda b, w: [""] * len(w))
    with pytest.raises(ValueError):
        srv.addImage("0", "x", 0.0, _crop(32))
    LocalServer(lambda b, w: [""] * len(w), accept_narrow=True).addImage("0", "x", 0.0, _crop(32))


def test_three_channel_crop_keeps_channel_one():
    b = Bucket(1.0, 4, (32, 64))
    img = np.zeros((32, 40, 3), np.uint8)
    img[:, :, 1] = 9
    b.addImgToBucket("0", "a", 0.0, img)
    assert b.imgs[0].shape == (32, 64, 1) and (b.imgs[0][:, :40] == 9).all()


def test_service_round_trip_with_stand_in_recogniser():
    """Crops of many widths from two clients come back to the right client and
    index; filler rows never reach a client."""
    seen = []

    def recog(batch, widths):
        seen.append((batch.shape, widths.tolist()))
        return [f"w{w}" for w in widths]

    srv = LocalServer(recog, bucket_size=4, bucket_max_time=0.0)
    p1, p2 = BatchLinePredictor(srv), BatchLinePredictor(srv)
    rng = np.random.default_rng(0)
    w1 = rng.integers(33, 600, 11).tolist()
    w2 = rng.integers(33, 600, 5).tolist()
    stop = threading.Event()
    th = threading.Thread(target=srv.run, kwargs={"stop": stop.is_set, "idle_sleep": 0.001})
    th.start()
    try:
        r1 = p1.predict_batch("b1", [_crop(w) for w in w1], give_up_after=20000)
        r2 = p2.predict_batch("b2", [_crop(w) for w in w2], give_up_after=20000)
    finally:
        stop.set()
        th.join()
    assert r1 == {i: f"w{w}" for i, w in enumerate(w1)}
    assert r2 == {i: f"w{w}" for i, w in enumerate(w2)}
    for shape, widths in seen:
        assert shape[0] == 4 and len(widths) == 4
        assert shape[2] % 32 == 0 and all(shape[2] - 32 < w <= shape[2] for w in widths)


class _FakeRecognizerFactory:
    """Picklable make_recognizer for ReplicaPool on CPU: the 'text' of a crop
    encodes its true width and the replica's device, so the test can check
    routing and delivery without a GPU."""

    def __call__(self, device):
        def rec(batch, widths):
            return [f"{device}:{int(w)}" for w in widths]
        return rec


def test_replica_pool_routes_whole_buckets_and_delivers():
    """Multi-replica recognise step (one worker process per device; whole
    width buckets per replica): every crop's result reaches its
    client, and a bucket always maps to the same replica."""
    import numpy as np

    from cnn_lstm_ctc_ocr_amd.server import LocalServer, ReplicaPool
    rng = np.random.default_rng(3)
    with ReplicaPool(["dev0", "dev1", "dev2"], _FakeRecognizerFactory()) as pool:
        srv = LocalServer(pool, bucket_size=4, bucket_max_time=0.0)
        cid, inq, outq = srv.register()
        widths = [int(w) for w in rng.integers(33, 400, 40)]
        for i, w in enumerate(widths):
            srv.addImage(cid, i, 0.0, rng.integers(0, 256, (32, w), dtype=np.uint8))
        for k in range(20):                              # the clock advances (bucket release, server.py:45,52)
            srv.flush_buckets(now=1e9 + k)
        srv.collect(block=True)
        got = {}
        while not outq.empty():
            imgid, txt = outq.get()
            got[imgid] = txt
        assert sorted(got) == list(range(len(widths)))
        for i, w in enumerate(widths):
            dev, tw = got[i].split(":")
            assert int(tw) == w
            bucket = (w - 1) // 32 - 1                      # buckets (w, w+32] from w = 32
            assert dev == f"dev{pool.replica_of(bucket)}"


class _FailingFactory:
    """make_recognizer that raises on one device (init failure) or returns a
    recognizer that kills its process / raises on a marked batch."""

    def __init__(self, mode):
        self.mode = mode

    def __call__(self, device):
        if self.mode == "init" and device == "dev1":
            raise RuntimeError("no such device")

        def rec(batch, widths):
            if self.mode == "die":
                import os
                os._exit(7)
            if self.mode == "raise" or (self.mode == "raise99" and int(widths[0]) == 99):
                raise ValueError("bad batch")
            return [str(int(w)) for w in widths]
        return rec


def test_replica_pool_reports_init_failure_with_rank():
    import pytest

    from cnn_lstm_ctc_ocr_amd.server import ReplicaError, ReplicaPool
    with pytest.raises(ReplicaError, match=r"replica 1 \(dev1\) failed to start: RuntimeError: no such device"):
        ReplicaPool(["dev0", "dev1"], _FailingFactory("init"), timeout=60)


def test_replica_pool_notices_a_dead_worker():
    import numpy as np
    import pytest

    from cnn_lstm_ctc_ocr_amd.server import ReplicaError, ReplicaPool
    pool = ReplicaPool(["dev0"], _FailingFactory("die"), timeout=60)
    pool.submit(0, 0, np.zeros((1, 32, 64, 1), np.uint8), [64])
    with pytest.raises(ReplicaError, match="replica 0 .* died with exit code 7"):
        pool.poll(block=True, timeout=60)
    pool.close()


def test_replica_pool_batch_error_names_the_replica():
    import numpy as np
    import pytest

    from cnn_lstm_ctc_ocr_amd.server import ReplicaError, ReplicaPool
    with ReplicaPool(["dev0", "dev1"], _FailingFactory("raise"), timeout=60) as pool:
        pool.submit(1, 5, np.zeros((1, 32, 64, 1), np.uint8), [64])
        with pytest.raises(ReplicaError, match="replica 1 failed on batch 5: ValueError: bad batch"):
            pool.poll(block=True, timeout=60)


def test_replica_pool_keeps_results_collected_before_an_error():
    """A poll() that raises for one replica's batch does not lose the results
    it had already collected from the other: the next poll() returns them."""
    import time

    import numpy as np
    import pytest

    from cnn_lstm_ctc_ocr_amd.server import ReplicaError, ReplicaPool
    with ReplicaPool(["dev0", "dev1"], _FailingFactory("raise99"), timeout=60) as pool:
        pool.submit(0, 1, np.zeros((1, 32, 64, 1), np.uint8), [64])
        pool.submit(1, 2, np.zeros((1, 32, 128, 1), np.uint8), [99])
        time.sleep(2.0)                                    # both replies queued before the poll
        with pytest.raises(ReplicaError, match="failed on batch 2"):
            pool.poll(block=True, timeout=60)
        got = pool.poll(block=True, timeout=60)
        assert got == [(1, ["64"])]
        assert not pool.assigned
