"""SyncBN (Trainer(sync_bn=True)): TRAIN-mode BatchNorm statistics and the
backward's two sums span all data-parallel ranks' batches, so N ranks compute
the single-device reference step (src/weinman/model.py:118-123's
batch_normalization over the whole batch, train.py:116-118's UPDATE_OPS) on the
union of their batches.

* the split C-ABI forms agree with the fused ones on one rank: ocrk_bn_moments +
  ocrk_bn_finalize_moments == ocrk_bn_finalize (same bits), and
  ocrk_bn_relu_pool_bwd_reduce + _apply == ocrk_bn_relu_pool_bwd for each of the
  path's pools and both storage types;
* two ranks (gloo carrying CUDA tensors on the box's one GPU), each half of a
  batch: the reduced gradient and the moving averages equal one process's on
  the whole batch -- and without sync_bn they do not."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
SIZES = (64, 64)
B, W = 32, 128


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,pool", [((4, 8, 40, 64), (2, 2, 2, 2)), ((4, 4, 33, 128), (2, 2, 2, 1)),
                                        ((4, 3, 31, 256), (3, 1, 3, 1)), ((2, 5, 12, 32), (2, 2, 2, 2))])
def test_split_bn_forms_match_the_fused_ones(cuda, dtype, shape, pool):
    from cnn_lstm_ctc_ocr_amd import _lib, kernels as K
    from cnn_lstm_ctc_ocr_amd._lib import ptr
    g = torch.Generator(device="cpu").manual_seed(11)
    Bn, H, Wd, C = shape
    M = Bn * H * Wd
    z = (torch.randn(shape, generator=g) * 2 + 0.5).to(dtype).to(cuda)
    tiles = (M + 127) // 128
    zf = z.float().reshape(M, C)
    stats = torch.zeros(tiles, 2, C, dtype=torch.float32, device=cuda)
    for t in range(tiles):                                # (sum, M2) per 128-row tile, as the epilogues leave them
        blk = zf[t * 128:(t + 1) * 128].double()
        stats[t, 0] = blk.sum(0).float()
        stats[t, 1] = ((blk - blk.mean(0)) ** 2).sum(0).float()
    mm0 = torch.rand(C, generator=g).to(cuda)
    mv0 = (torch.rand(C, generator=g) + 0.5).to(cuda)
    mm1, mv1, mm2, mv2 = mm0.clone(), mv0.clone(), mm0.clone(), mv0.clone()
    mean, invstd = K.bn_finalize(stats, M, C, 1e-3, 0.99, mm1, mv1)
    moments = torch.empty(3 * C + 1, dtype=torch.float64, device=cuda)
    nb = _lib.lib().ocrk_bn_finalize_workspace_size(tiles, C)
    ws = torch.empty(nb, dtype=torch.uint8, device=cuda)
    _lib.call("ocrk_bn_moments", ptr(stats), tiles, 128, M, C, ptr(moments), ptr(ws), nb, K._stream(stats))
    mean2 = torch.empty_like(mean)
    invstd2 = torch.empty_like(mean)
    _lib.call("ocrk_bn_finalize_moments", ptr(moments), C, 1e-3, 0.99, ptr(mean2), ptr(invstd2), ptr(mm2), ptr(mv2),
              K._stream(stats))
    torch.cuda.synchronize()
    assert torch.equal(mean, mean2) and torch.equal(invstd, invstd2)
    assert torch.equal(mm1, mm2) and torch.equal(mv1, mv2)
    assert moments[3 * C].item() == M

    kh, kw, sh, sw = pool
    Ho, Wo = (H - kh) // sh + 1, (Wd - kw) // sw + 1
    dp = torch.randn(Bn, Ho, Wo, C, generator=g).to(dtype).to(cuda)
    gamma = (torch.rand(C, generator=g) + 0.5).to(cuda)
    beta = (torch.randn(C, generator=g) * 0.1).to(cuda)
    dg1, db1, dbias1 = (torch.zeros(C, device=cuda) for _ in range(3))
    dz1 = K.bn_relu_pool_bwd(z, dp, mean, invstd, gamma, beta, pool, False, dg1, db1, dbias=dbias1)
    dg2, db2, dbias2 = (torch.zeros(C, device=cuda) for _ in range(3))
    dsum = torch.empty(2 * C, dtype=torch.float32, device=cuda)
    count = torch.full((1,), float(M), dtype=torch.float64, device=cuda)
    nbw = _lib.lib().ocrk_bn_bwd_workspace_size(Bn, H, Wd, C)
    wsb = torch.empty(nbw, dtype=torch.uint8, device=cuda)
    dz2 = torch.empty_like(z)
    args = (ptr(z), ptr(dp), Bn, H, Wd, C, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta), kh, kw, sh, sw, 0)
    _lib.call("ocrk_bn_relu_pool_bwd_reduce", *args, ptr(dg2), ptr(db2), 1, ptr(dsum), ptr(wsb), nbw,
              K.dtype_code(dtype), K._stream(z))
    _lib.call("ocrk_bn_relu_pool_bwd_apply", *args, ptr(dsum), ptr(count), ptr(dz2), ptr(dbias2), 1, None,
              ptr(wsb), nbw, K.dtype_code(dtype), K._stream(z))
    torch.cuda.synchronize()
    assert torch.equal(dg1, dg2) and torch.equal(db1, db2)
    # the apply pass scales dsum by pixels / count (= 1 here): same bits
    assert torch.equal(dz1, dz2) and torch.equal(dbias1, dbias2)


def _batch():
    rng = np.random.default_rng(91)
    img = rng.integers(0, 256, (B, 32, W, 1), dtype=np.uint8)
    labels = [list(rng.integers(0, 95, int(rng.integers(2, 8)))) for _ in range(B)]
    return img, labels


def _grads(store, tr, img, labels, device):
    tr.loss_and_grads(torch.from_numpy(img).to(device), np.full(img.shape[0], W, np.int32), labels)
    scale = tr.reduce_gradients()
    torch.cuda.synchronize()
    return store.flat_grad.cpu().numpy() * scale, store.flat_stats.cpu().numpy()


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OCRK_LSTM_PERSISTENT="0")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    dev = torch.device("cuda:0")
    img, labels = _batch()
    half = B // world
    sl = slice(rank * half, (rank + 1) * half)
    for sync in (True, False):
        store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=SIZES, dtype=torch.float32), device=dev, seed=5)
        tr = Trainer(store, sync_bn=sync)
        g, st = _grads(store, tr, img[sl], labels[sl], dev)
        tr.check_status()
        np.save(os.path.join(outdir, f"g{int(sync)}_{rank}.npy"), g)
        np.save(os.path.join(outdir, f"s{int(sync)}_{rank}.npy"), st)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sync_bn_step_equals_the_whole_batch_on_one_device(cuda, tmp_path):
    import torch.multiprocessing as mp
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=SIZES, dtype=torch.float32), device=cuda, seed=5)
    img, labels = _batch()
    want, want_st = _grads(store, Trainer(store), img, labels, cuda)
    g0, g1 = np.load(tmp_path / "g1_0.npy"), np.load(tmp_path / "g1_1.npy")
    np.testing.assert_array_equal(g0, g1)
    # fp32 (exact products); the two ranks' BN sums are merged in another order
    # than one process's, and the BN backward amplifies that rounding ~100x
    err = np.linalg.norm(g0 - want) / np.linalg.norm(want)
    assert err < 1e-4, err
    s0, s1 = np.load(tmp_path / "s1_0.npy"), np.load(tmp_path / "s1_1.npy")
    np.testing.assert_array_equal(s0, s1)              # every rank's moving averages are the union's
    np.testing.assert_allclose(s0, want_st, rtol=1e-5, atol=1e-6)
    # per-rank statistics (no sync_bn) are a different step: the check above discriminates
    n0 = np.load(tmp_path / "g0_0.npy")
    assert np.linalg.norm(n0 - want) / np.linalg.norm(want) > 1e-3
    assert not np.allclose(np.load(tmp_path / "s0_0.npy"), want_st, rtol=1e-5, atol=1e-6)
