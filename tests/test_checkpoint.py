"""TF1 TensorBundle checkpoints (train.py / validate.py / test.py Saver paths)."""
import os
import struct

import numpy as np
import pytest
import torch

from cnn_lstm_ctc_ocr_amd import checkpoint as C
from cnn_lstm_ctc_ocr_amd.tfrecord import masked_crc32c


def test_crc32c_check_value():
    from cnn_lstm_ctc_ocr_amd.tfrecord import crc32c, crc32c_py
    assert crc32c(b"123456789") == 0xE3069283 == crc32c_py(b"123456789")


def test_bundle_round_trip_many_entries_and_dtypes(tmp_path):
    rng = np.random.default_rng(0)
    t = {f"rnn/bdrnn{i % 3}/fw/lstm_cell/kernel_{i:03d}": rng.standard_normal((i % 5 + 1, 7)).astype(np.float32)
         for i in range(60)}                         # > restart interval, > one 4 KiB block
    t["global_step"] = np.array(1234, np.int64)
    t["convnet/conv1/kernel"] = rng.standard_normal((3, 3, 1, 32)).astype(np.float32)
    t["ints"] = np.arange(10, dtype=np.int32)
    t["halfs"] = np.linspace(0, 1, 9).astype(np.float16)
    prefix = str(tmp_path / "model.ckpt-7")
    C.write_bundle(prefix, t)
    got = C.read_bundle(prefix, verify=True)
    assert set(got) == set(t)
    for k in t:
        assert got[k].dtype == t[k].dtype and got[k].shape == t[k].shape
        np.testing.assert_array_equal(got[k], t[k])


def _hand_table(pairs):
    """An SSTable built straight from the LevelDB format description, with
    choices the writer does not make (one restart per entry, no prefix sharing)."""
    def varint(v):
        out = bytearray()
        while True:
            b, v = v & 0x7F, v >> 7
            out.append(b | (0x80 if v else 0))
            if not v:
                return bytes(out)

    def block(entries):
        body = bytearray()
        restarts = []
        for k, v in entries:
            restarts.append(len(body))
            body += varint(0) + varint(len(k)) + varint(len(v)) + k + v
        body += b"".join(struct.pack("<I", r) for r in (restarts or [0]))
        body += struct.pack("<I", len(restarts or [0]))
        return bytes(body)

    out = bytearray()

    def put(b):
        off = len(out)
        out.extend(b + b"\x00" + struct.pack("<I", masked_crc32c(b + b"\x00")))
        return varint(off) + varint(len(b))

    data_h = put(block(pairs))
    meta_h = put(block([]))
    index_h = put(block([(pairs[-1][0], data_h)]))
    footer = meta_h + index_h
    out.extend(footer + b"\x00" * (40 - len(footer)) + struct.pack("<Q", 0xDB4775248B80FB57))
    return bytes(out)


def test_reader_on_hand_built_table(tmp_path):
    pairs = [(b"", b"hdr"), (b"a/b", b"1"), (b"a/bc", b"22"), (b"b", b"333")]
    p = tmp_path / "t.index"
    p.write_bytes(_hand_table(pairs))
    assert C.read_table(str(p), verify=True) == pairs


def test_read_bundle_rejects_corruption(tmp_path):
    prefix = str(tmp_path / "m")
    C.write_bundle(prefix, {"x": np.arange(100, dtype=np.float32)})
    data = prefix + ".data-00000-of-00001"
    raw = bytearray(open(data, "rb").read())
    raw[5] ^= 0xFF
    open(data, "wb").write(raw)
    with pytest.raises(ValueError):
        C.read_bundle(prefix, verify=True)


def test_latest_checkpoint_parses_state_file(tmp_path):
    (tmp_path / "checkpoint").write_text('model_checkpoint_path: "model.ckpt-300"\n'
                                         'all_model_checkpoint_paths: "model.ckpt-200"\n'
                                         'all_model_checkpoint_paths: "model.ckpt-300"\n')
    assert C.latest_checkpoint(str(tmp_path)) == str(tmp_path / "model.ckpt-300")
    with pytest.raises(RuntimeError):
        C.latest_checkpoint(str(tmp_path / "nope"))


@pytest.mark.parametrize("cell,sizes", [("lstm", (32, 32)), ("gru", (64, 32))])
def test_store_save_restore_with_adam_slots(tmp_path, cell, sizes):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    cfg = ModelConfig(cell=cell, rnn_sizes=sizes, dtype=torch.float32)
    a = ParamStore(cfg, device="cpu", seed=1)
    a.stats["convnet/conv2/batch_norm/moving_mean"].fill_(0.25)
    ta = Trainer(a, global_step=42)
    ta.m.uniform_()
    ta.v.uniform_()
    with pytest.raises(ValueError, match="trainer is at step 42"):
        C.save(a, str(tmp_path), global_step=41, trainer=ta)      # one source for the step
    prefix = C.save(a, str(tmp_path), trainer=ta)
    assert os.path.basename(prefix) == "model.ckpt-42"
    b = ParamStore(cfg, device="cpu", seed=2)
    tb = Trainer(b)
    C.restore(b, str(tmp_path), trainer=tb)
    for k, v in a.state_dict().items():
        np.testing.assert_array_equal(b.state_dict()[k], v, err_msg=k)
    assert tb.global_step == 42
    for n, p in a.params.items():
        _, off, _ = a.offsets[n]
        assert torch.equal(tb.m[off:off + p.numel()], ta.m[off:off + p.numel()])
        assert torch.equal(tb.v[off:off + p.numel()], ta.v[off:off + p.numel()])
    names = C.read_bundle(prefix)
    assert "rnn/bdrnn1/fw/" + ("lstm_cell/kernel" if cell == "lstm" else "gru_cell/gates/kernel") in names
    assert "convnet/conv1/kernel/Adam_1" in names and names["global_step"] == 42


def test_saved_adam_powers_follow_tf1_finish():
    """TF1 AdamOptimizer holds beta^(t+1) after t updates (created as
    beta, multiplied by beta in every _finish). A checkpoint written at t = 0
    must not hold 1.0 (TF would compute lr_t = lr * 0 / 0)."""
    import tempfile

    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    assert C.adam_power(0.9, 0) == np.float32(0.9)
    p = np.float32(0.999)
    for _ in range(3):
        p = np.float32(p * np.float32(0.999))
    assert C.adam_power(0.999, 3) == p
    cfg = ModelConfig(cell="lstm", rnn_sizes=(32, 32), dtype=torch.float32)
    store = ParamStore(cfg, device="cpu", seed=1)
    tr = Trainer(store)
    tr.global_step = 5
    with tempfile.TemporaryDirectory() as d:
        t = C.read_bundle(C.save(store, d, global_step=5, trainer=tr))
    np.testing.assert_allclose(t["beta1_power"], 0.9 ** 6, rtol=1e-6)
    np.testing.assert_allclose(t["beta2_power"], 0.999 ** 6, rtol=1e-6)
