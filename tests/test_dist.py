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


def _bucket_worker(rank, world, port, out):
    """The Trainer's bucketed all-reduce over a real ParamStore flat layout:
    the recurrent bucket is started mid-"backward" (the hook), the conv
    bucket after it; the result and the Adam grad_scale must equal the mean
    gradient of the concatenated batch."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(32, 32), dtype=torch.float32), device="cpu", seed=1)
    tr = Trainer(store)
    g = store.flat_grad
    split = tr.buckets.split
    rng = np.random.default_rng(500 + rank)
    rnn_part = torch.from_numpy(rng.standard_normal(g.numel() - split).astype(np.float32))
    conv_part = torch.from_numpy(rng.standard_normal(split).astype(np.float32))
    g[split:].copy_(rnn_part)                   # the recurrent + logits backward wrote its bucket ...
    tr.buckets.rnn_ready()                      # ... the hook starts its all-reduce
    g[:split].copy_(conv_part)                  # the conv tower's backward
    scale = tr.reduce_gradients()
    out[rank] = (g.numpy().copy(), scale, split, store.offsets["rnn/bdrnn1/fw/lstm_cell/kernel"][1])
    dist.barrier()
    dist.destroy_process_group()


def test_bucketed_allreduce_over_paramstore_layout():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bucket_worker, args=(world, port, out), nprocs=world, join=True)
    g0, s0, split, first_rnn = out[0]
    g1, s1, _, _ = out[1]
    assert split == first_rnn                   # the conv tower sits in front of the recurrent bucket
    parts = []
    for r in range(world):
        rng = np.random.default_rng(500 + r)
        rnn = rng.standard_normal(g0.size - split).astype(np.float32)
        conv = rng.standard_normal(split).astype(np.float32)
        parts.append(np.concatenate([conv, rnn]))
    total = sum(parts)
    np.testing.assert_allclose(g0, total, rtol=1e-6)
    np.testing.assert_allclose(g1, total, rtol=1e-6)
    assert s0 == s1 == 0.5
    # Adam (the kernel receives grad_scale) on the summed gradient == Adam on the global mean
    mean = sum(p.astype(np.float64) for p in parts) / world
    p_ = np.zeros_like(mean)
    a, _, _ = G.adam_update(p_.copy(), total.astype(np.float64) * s0, np.zeros_like(mean), np.zeros_like(mean),
                            1e-4, 1)
    b, _, _ = G.adam_update(p_.copy(), mean, np.zeros_like(mean), np.zeros_like(mean), 1e-4, 1)
    np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-12)


def _status_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cnn_lstm_ctc_ocr_amd.train import or_allreduce_status
    # rank 0: CTC_INFEASIBLE | LSTM_FWD_TIMEOUT; rank 1: LSTM_BWD_TIMEOUT (include/ocrk.h)
    word = torch.tensor([0x12 if rank == 0 else 0x20], dtype=torch.int32)
    or_allreduce_status(word)
    out[rank] = int(word[0])
    dist.barrier()
    dist.destroy_process_group()


def test_status_word_is_or_reduced_over_ranks():
    """The device status word is a bitmask: the data-parallel reduction keeps
    every rank's bits (a MAX of the words would leave 0x20 on both ranks and
    lose the infeasible-label and forward-timeout bits)."""
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_status_worker, args=(2, port, out), nprocs=2, join=True)
    assert out[0] == out[1] == 0x32


# ------------------------------------------------------------------ SyncBN
def _bn_shard(rank):
    rng = np.random.default_rng(300 + rank)
    x = rng.standard_normal((2 + rank, 3, 50, 8)) * 1.5 + 0.3     # unequal shards: 300 and 450 pixels
    dy = rng.standard_normal(x.shape)
    return x, dy


def _moments(x, tile_rows=128):
    """The additive per-rank summary ocrk_bn_moments leaves (bn.hip): per-tile
    (sum, M2) merged as S = sum x, Q = sum_t s_t^2 / n_t, W2 = sum_t M2_t, and M."""
    v = x.reshape(-1, x.shape[-1])
    S, Q, W2 = (np.zeros(v.shape[1]) for _ in range(3))
    for t0 in range(0, v.shape[0], tile_rows):
        blk = v[t0:t0 + tile_rows]
        s = blk.sum(0)
        S += s
        Q += s * s / blk.shape[0]
        W2 += ((blk - blk.mean(0)) ** 2).sum(0)
    return np.concatenate([S, Q, W2, [v.shape[0]]])


def _syncbn_worker(rank, world, port, out):
    """Host protocol of Trainer(sync_bn=True) per BN layer: SUM all-reduce of
    the moments, finalize (bn_final_channel); backward SUM all-reduce of
    (sum dy, sum dy*xhat), dz over the union's count."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, dy = _bn_shard(rank)
    C = x.shape[-1]
    mom = torch.from_numpy(_moments(x))
    dist.all_reduce(mom, op=dist.ReduceOp.SUM)
    S, Q, W2, n = mom[:C].numpy(), mom[C:2 * C].numpy(), mom[2 * C:3 * C].numpy(), mom[3 * C].item()
    mu = S / n
    var = np.maximum(W2 + Q - S * mu, 0.0) / n
    inv = 1.0 / np.sqrt(var + G.BN_EPS)
    xhat = (x - mu) * inv
    dsum = torch.from_numpy(np.concatenate([dy.sum((0, 1, 2)), (dy * xhat).sum((0, 1, 2))]))
    dist.all_reduce(dsum, op=dist.ReduceOp.SUM)
    gamma = np.linspace(0.5, 1.5, C)
    dx = gamma * inv * (dy - dsum[:C].numpy() / n - xhat * dsum[C:].numpy() / n)
    out[rank] = (mu, var, dx)
    dist.barrier()
    dist.destroy_process_group()


def test_sync_bn_protocol_matches_the_union_batch():
    """Two ranks with unequal shards: the all-reduced moments give the union's
    batch mean / variance and the split backward gives the union's dx rows
    (oracle bn_train / bn_bwd on the concatenated batch, model.py:118-123)."""
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_syncbn_worker, args=(world, port, out), nprocs=world, join=True)
    xs, dys = zip(*[_bn_shard(r) for r in range(world)])
    x, dy = np.concatenate(xs), np.concatenate(dys)
    C = x.shape[-1]
    gamma = np.linspace(0.5, 1.5, C)
    _, mean, var, _, cache = G.bn_train(x, gamma, np.zeros(C))
    dx, _, _ = G.bn_bwd(dy, cache, gamma)
    rows = np.cumsum([0] + [s.shape[0] for s in xs])
    for r in range(world):
        mu_r, var_r, dx_r = out[r]
        np.testing.assert_allclose(mu_r, mean, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(var_r, var, rtol=1e-12)
        np.testing.assert_allclose(dx_r, dx[rows[r]:rows[r + 1]], rtol=1e-10, atol=1e-12)


def _syncbn_group_worker(rank, world, port, out):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(32, 32), dtype=torch.float32), device="cpu", seed=1)
    tr = Trainer(store, sync_bn=True)           # built BEFORE the process group exists
    before = tr._bn_group()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    after = tr._bn_group()
    other = Trainer(store)                      # a second trainer on the same (shared) store
    out[rank] = (before is None, after is dist.group.WORLD, other._bn_group() is None,
                 tr._bn_group() is dist.group.WORLD, store.bn_group is None)
    dist.barrier()
    dist.destroy_process_group()


def test_sync_bn_group_resolved_when_the_step_runs():
    """Trainer(sync_bn=True) built before init_process_group must
    still synchronise once the group exists (the group is resolved per step,
    not captured at construction), and a later Trainer on the same ParamStore
    must not switch it off (the setting lives on the Trainer; the store only
    carries it for the duration of that Trainer's own forward + backward)."""
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_syncbn_group_worker, args=(2, port, out), nprocs=2, join=True)
    assert out[0] == out[1] == (True, True, True, True, True)
