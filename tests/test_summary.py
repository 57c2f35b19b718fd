"""JSONL scalar summaries (the reference's tf.summary scalars,
train.py:139 learning_rate, test.py:100-102 loss / label_error /
sequence_error) -- host logic on the CPU."""
import torch

from cnn_lstm_ctc_ocr_amd import summary


def test_writer_records_in_step_order(tmp_path):
    p = tmp_path / "m.jsonl"
    with summary.SummaryWriter(str(p)) as w:
        w.scalars(1, loss=torch.tensor(2.5), learning_rate=1e-4)
        w.scalars(2, loss=torch.tensor([1.25]), label_error=0.5)
    recs = summary.read(str(p))
    assert [r["step"] for r in recs] == [1, 2]
    assert recs[0]["loss"] == 2.5 and recs[0]["learning_rate"] == 1e-4
    assert recs[1]["loss"] == 1.25 and recs[1]["label_error"] == 0.5
    assert all("wall_time" in r for r in recs)


def test_only_rank_zero_writes(tmp_path):
    p = tmp_path / "r1.jsonl"
    w = summary.SummaryWriter(str(p), rank=1)
    w.scalars(1, loss=1.0)
    w.close()
    assert not p.exists()


def test_trainer_summarizes_every_n_steps(tmp_path):
    """Trainer.summarize (called by step() after the update): every
    `summary_every` steps, learning_rate of the step (exponential_decay,
    train.py:120-126), its loss and the crops/s since the last record."""
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(32, 32), dtype=torch.float32), device="cpu", seed=1)
    p = tmp_path / "train.jsonl"
    w = summary.SummaryWriter(str(p))
    tr = Trainer(store, summary=w, summary_every=2, decay_steps=4)
    for i in range(5):
        lr = tr.learning_rate()
        tr.global_step += 1                      # what apply_gradients does
        tr.summarize(torch.tensor(float(10 - i)), lr, batch=8)
    w.close()
    recs = summary.read(str(p))
    assert [r["step"] for r in recs] == [2, 4]
    assert recs[0]["loss"] == 9.0 and recs[1]["loss"] == 7.0
    assert abs(recs[1]["learning_rate"] - 1e-4 * 0.9 ** (3 / 4)) < 1e-12
    assert recs[0]["crops_per_sec"] > 0


def test_writer_evaluates_deferred_values(tmp_path):
    """A callable value (the trainer's device-timed crops/s) is evaluated when
    the record is written, not when it is queued."""
    p = tmp_path / "d.jsonl"
    box = {"v": 1.0}
    with summary.SummaryWriter(str(p)) as w:
        w.scalars(3, rate=lambda: box["v"] * 2)
        box["v"] = 5.0
    assert summary.read(str(p))[0]["rate"] in (2.0, 10.0)
