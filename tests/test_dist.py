"""Data-parallel host logic on CPU with gloo (world_size 2): the flat gradient
all-reduce + 1/world scale reproduces the single-process gradient of the
concatenated batch (the loss is a batch mean, model.py:228)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_graph as G


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard(rank):
    rng = np.random.default_rng(100 + rank)
    T, B, C = 12, 3, 96
    logits = rng.standard_normal((T, B, C)).astype(np.float64)
    labels = [list(rng.integers(0, 95, 3)) for _ in range(B)]
    seq = np.array([12, 10, 9])
    return logits, labels, seq


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cnn_lstm_ctc_ocr_amd.train import allreduce_mean_scale
    logits, labels, seq = _shard(rank)
    _, g = G.ctc_loss(logits, labels, seq)
    flat = torch.from_numpy((g / logits.shape[1]).reshape(-1).copy())   # d mean-loss / d logits
    scale = allreduce_mean_scale(flat)
    out[rank] = (flat * scale).numpy()
    dist.barrier()
    dist.destroy_process_group()


def test_dp_allreduce_mean_matches_global_batch():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    # single process: gradient of the mean loss over the concatenated batch,
    # evaluated per shard position (logits of each shard are distinct inputs)
    full = []
    for r in range(world):
        logits, labels, seq = _shard(r)
        _, g = G.ctc_loss(logits, labels, seq)
        full.append(g / (logits.shape[1] * world))
    summed = sum(f.reshape(-1) for f in full)
    np.testing.assert_allclose(out[0], summed, rtol=1e-12)
    np.testing.assert_allclose(out[1], summed, rtol=1e-12)


def test_single_process_scale_is_one():
    from cnn_lstm_ctc_ocr_amd.train import allreduce_mean_scale
    t = torch.ones(4)
    assert allreduce_mean_scale(t) == 1.0 and torch.equal(t, torch.ones(4))
