"""The data-parallel exchange of the train step with RCCL really executing
(VERDICT r5 "next" #2): the reference's loss is a batch mean
(src/weinman/model.py:224-229), so the exchange is a SUM all-reduce of the flat
gradient followed by Adam's 1/world. The box has one GPU (RCCL refuses two ranks
on one device), so the exchange is FORCED at world 1 (GradBuckets(force=True)):
the recurrent + logits bucket's all-reduce starts from the hook on the conv
tower's output gradient on the comm stream, beside the conv backward, the conv
bucket follows, the status word is OR-reduced, and the next step's persistent
loops start behind the join -- the C4 step's whole ordering, on the bench's own
route (bf16, LSTM 512/512, persistent loops, side-stream weight gradients,
B = 256, 32x256 crops).

Three steps through torch.distributed (backend "nccl" = RCCL) and three through
the C ABI (libocrk_comm.so, include/ocrk_comm.h) must leave the parameters, Adam
moments and BN moving statistics BIT-identical to three undistributed steps (the
sum over one rank is the identity and every kernel reduces in a fixed order),
with no status bit (no *_TIMEOUT from a hand-off wait beside a collective).
What one GPU cannot show: the multi-rank sum itself (tests/test_dist.py and
test_gpu_dist.py check it over gloo) -- the driver's 8-GPU run is its RCCL test."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
B, W, STEPS = 256, 256, 3


def _run(mode, port, outdir):
    """mode: "plain" (no exchange), "nccl" (torch.distributed RCCL, forced at world 1)
    or "capi" (the libocrk_comm.so communicator, forced)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    import bench
    import torch.distributed as dist
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd import kernels as K
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    dev = torch.device("cuda:0")
    comm = None
    if mode == "nccl":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    elif mode == "capi":
        from cnn_lstm_ctc_ocr_amd import comm as C
        comm = C.Communicator(1, 0, C.unique_id(), 0)
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=torch.bfloat16), device=dev, seed=5)
    assert K.lstm_persistent_ok(B, 512, torch.bfloat16)
    tr = Trainer(store, comm=comm, force_exchange=mode != "plain")
    calls = {"hook": 0, "sum": 0}
    hook, sum_ = tr.buckets.rnn_ready, tr.buckets._sum_

    def counted_hook(*a):
        calls["hook"] += 1
        return hook(*a)

    def counted_sum(*a, **k):
        calls["sum"] += 1
        return sum_(*a, **k)
    tr.buckets.rnn_ready, tr.buckets._sum_ = counted_hook, counted_sum
    rng = np.random.default_rng(77)
    batches = [bench.synthetic_batch(rng, B, W, 125, dev) for _ in range(STEPS)]
    losses = [float(tr.step(*b)) for b in batches]
    assert tr.buckets.work is None
    tr.check_status()                                  # no hand-off wait gave up beside the collective
    torch.cuda.synchronize()
    np.savez(os.path.join(outdir, f"{mode}.npz"), flat=store.flat.cpu().numpy(), m=tr.m.cpu().numpy(),
             v=tr.v.cpu().numpy(), stats=store.flat_stats.cpu().numpy(), losses=np.array(losses),
             hook=calls["hook"], sums=calls["sum"], world=tr.world_size())
    if comm is not None:
        comm.close()
    if mode == "nccl":
        dist.destroy_process_group()


def _worker(rank, modes, port, outdir):
    for m in modes:
        _run(m, port, outdir)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_forced_rccl_exchange_train_steps_bit_identical(cuda, tmp_path):
    import torch.multiprocessing as mp
    # one fresh process for the distributed runs (no process group left in pytest's)
    mp.start_processes(_worker, args=(("nccl", "capi"), _port(), str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    _run("plain", _port(), str(tmp_path))
    ref = np.load(tmp_path / "plain.npz")
    assert int(ref["hook"]) == 0 and int(ref["sums"]) == 0
    for mode in ("nccl", "capi"):
        got = np.load(tmp_path / f"{mode}.npz")
        assert int(got["world"]) == 1
        # per step: the hook's recurrent bucket + the conv bucket (the status OR is separate)
        assert int(got["hook"]) == STEPS and int(got["sums"]) == 2 * STEPS, (mode, got["hook"], got["sums"])
        for k in ("flat", "m", "v", "stats", "losses"):
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{mode}: {k}")
