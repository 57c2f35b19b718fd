"""Per-op parity of the HIP kernels against the oracle / numpy (fp32 within
float tolerances; index work bit-exact)."""
import numpy as np
import pytest
import torch

from oracle import ref_graph as G

pytestmark = pytest.mark.gpu


def _t(x, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    return t.to(dtype) if dtype is not None else t


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


# --------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False)])
@pytest.mark.parametrize("M,N,K", [(200, 96, 160), (64, 512, 1000), (296, 40, 72)])
def test_gemm_modes(cuda, dtype, ta, tb, M, N, K):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    B = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    if dtype == torch.bfloat16:   # compare against the bf16-rounded operands
        A = torch.from_numpy(A).bfloat16().float().numpy()
        B = torch.from_numpy(B).bfloat16().float().numpy()
    ref = (A.T if ta else A).astype(np.float64) @ (B.T if tb else B).astype(np.float64) + bias
    # fp32 operands run on the bf16x3 split (mfma_util.h: ~2^-16 relative per product,
    # f32 accumulation): 2e-5 relative L2 on standard-normal operands; bf16 operands
    # are exact products with f32 accumulation
    tol = 2e-5 if dtype == torch.float32 else 2e-6
    out = Kn.gemm(_t(A, cuda, dtype), _t(B, cuda, dtype), trans_a=ta, trans_b=tb, bias=_t(bias, cuda))
    assert _rel(out.cpu().numpy(), ref) < tol
    out = Kn.gemm(_t(A, cuda, dtype), _t(B, cuda, dtype), trans_a=ta, trans_b=tb, bias=_t(bias, cuda), relu=True,
                  splits=3)
    assert _rel(out.cpu().numpy(), np.maximum(ref, 0)) < tol


def test_gemm_accumulate_and_bf16_out(cuda):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(0)
    A = rng.standard_normal((128, 64)).astype(np.float32)
    B = rng.standard_normal((64, 32)).astype(np.float32)
    C = rng.standard_normal((128, 32)).astype(np.float32)
    c = _t(C, cuda)
    Kn.gemm(_t(A, cuda), _t(B, cuda), out=c, accumulate=True)
    np.testing.assert_allclose(c.cpu().numpy(), C + A @ B, rtol=1e-4, atol=1e-4)     # bf16x3 fp32 products
    ob = Kn.gemm(_t(A, cuda), _t(B, cuda), out_dtype=torch.bfloat16)
    np.testing.assert_allclose(ob.float().cpu().numpy(), A @ B, rtol=1e-2, atol=1e-2)


# --------------------------------------------------------------------- conv
@pytest.mark.parametrize("H,W", [(32, 40), (32, 259), (10, 600)])
def test_conv1_fwd_and_wgrad(cuda, H, W):
    """Row-strip workgroups: one strip, a second strip holding one pixel,
    three strips and a partial row group (Ho = 8 = 6 + 2)."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (3, H, W)).astype(np.uint8)
    w = rng.standard_normal((3, 3, 1, 32)).astype(np.float32)
    b = rng.standard_normal(32).astype(np.float32)
    x = G.preprocess(img)[..., None]
    ref = G.relu(G.conv2d(x, w, b, "valid"))
    y = Kn.conv1_fwd(_t(img, cuda), _t(w, cuda), _t(b, cuda), torch.float32)
    np.testing.assert_allclose(y.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    dz = rng.standard_normal(ref.shape).astype(np.float32)
    _, dw_ref, db_ref = G.conv2d_bwd(x, w, dz, "valid", need_dx=False)
    dw = torch.zeros(3, 3, 1, 32, device=cuda)
    db = torch.zeros(32, device=cuda)
    Kn.conv1_bwd_weight(_t(img, cuda), _t(dz, cuda), dw, db, accumulate=False)
    np.testing.assert_allclose(dw.cpu().numpy(), dw_ref, rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(db.cpu().numpy(), db_ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("cin,cout,relu", [(32, 32, False), (64, 128, True), (256, 256, False)])
def test_conv3x3_fwd_bwd(cuda, cin, cout, relu):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(cin + cout)
    x = rng.standard_normal((2, 5, 13, cin)).astype(np.float32)
    w = (rng.standard_normal((3, 3, cin, cout)) / np.sqrt(9 * cin)).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    z = G.conv2d(x, w, b, "same")
    ref = G.relu(z) if relu else z
    w_nk = Kn.permute3(_t(w, cuda), 9 * cin, cout, 1, torch.float32).view(cout, 9 * cin)
    w_bwd = Kn.permute3(_t(w, cuda), 9, cin, cout, torch.float32).view(cin, 9 * cout)
    M = 2 * 5 * 13
    stats = torch.empty(Kn.conv_stats_tiles(M), 2, cout, device=cuda)
    y = Kn.conv3x3_fwd(_t(x, cuda), w_nk, _t(b, cuda), relu, stats=stats)
    np.testing.assert_allclose(y.cpu().numpy(), ref, rtol=1e-4, atol=1e-4)
    mean, invstd = Kn.bn_finalize(stats, M, cout, 1e-3, 0.99)
    np.testing.assert_allclose(mean.cpu().numpy(), ref.reshape(-1, cout).mean(0), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(invstd.cpu().numpy(), 1 / np.sqrt(ref.reshape(-1, cout).var(0) + 1e-3), rtol=1e-4)
    dy = rng.standard_normal(z.shape).astype(np.float32)
    dx_ref, dw_ref, _ = G.conv2d_bwd(x, w, dy, "same")
    mask = rng.standard_normal(x.shape).astype(np.float32)
    dbias = torch.full((cin,), 0.25, device=cuda)
    dx = Kn.conv3x3_bwd_data(_t(dy, cuda), w_bwd, relu_mask=_t(mask, cuda), dbias=dbias, accumulate=True)
    np.testing.assert_allclose(dx.cpu().numpy(), dx_ref * (mask > 0), rtol=1e-4, atol=1e-4)
    # fused bias gradient of the producing layer = column sums of the masked dx
    np.testing.assert_allclose(dbias.cpu().numpy(), 0.25 + (dx_ref * (mask > 0)).reshape(-1, cin).sum(0),
                               rtol=1e-4, atol=1e-3)
    dw = torch.zeros(3, 3, cin, cout, device=cuda)
    Kn.conv3x3_bwd_weight(_t(x, cuda), _t(dy, cuda), dw, accumulate=False)
    np.testing.assert_allclose(dw.cpu().numpy(), dw_ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("B,H,W,cin,cout", [(4, 15, 127, 64, 64), (4, 7, 126, 128, 128), (6, 3, 125, 256, 256),
                                             (3, 5, 9, 64, 32)])
def test_f32_exact_conv_on_nt_ring(cuda, ocrk_opts, B, H, W, cin, cout):
    """Exact-mode fp32 convolutions (the fp32 Trainer's conv tower) on the NT
    ring's EXACT variants -- v_mfma_f32_16x16x4_f32 (default) and six bf16
    products of a three-way split (option NT_F32_X6=1) -- against
    the float64 graph and against the generic engine (NT_F32_EXACT=0): forward
    with the BN-statistics epilogue, the unmasked data gradient, and the masked
    one (the ReLU mask of the producing layer, fp32, in the epilogue) with the
    producing layer's fused bias gradient."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(B * cin + W)
    x = rng.standard_normal((B, H, W, cin)).astype(np.float32)
    w = (rng.standard_normal((3, 3, cin, cout)) / np.sqrt(9 * cin)).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    z = G.conv2d(x.astype(np.float64), w.astype(np.float64), b.astype(np.float64), "same")
    dy = rng.standard_normal(z.shape).astype(np.float32)
    dx_ref, _, _ = G.conv2d_bwd(x.astype(np.float64), w.astype(np.float64), dy.astype(np.float64), "same")
    mask = rng.standard_normal(x.shape).astype(np.float32)
    w_nk = Kn.permute3(_t(w, cuda), 9 * cin, cout, 1, torch.float32).view(cout, 9 * cin)
    w_bwd = Kn.permute3(_t(w, cuda), 9, cin, cout, torch.float32).view(cin, 9 * cout)
    M = B * H * W
    outs = {}
    # 2: the NT ring's six-product split (opt-in), 1: its f32 MFMA form (default), 0: the generic engine
    for mode in (2, 1, 0):
        ocrk_opts("NT_F32_EXACT", int(mode > 0))
        ocrk_opts("NT_F32_X6", int(mode == 2))
        with Kn.f32_exact():
            stats = torch.empty(Kn.conv_stats_tiles(M), 2, cout, device=cuda)
            y = Kn.conv3x3_fwd(_t(x, cuda), w_nk, _t(b, cuda), False, stats=stats)
            dx = Kn.conv3x3_bwd_data(_t(dy, cuda), w_bwd)
            dbias = torch.full((cin,), 0.25, device=cuda)
            dxm = Kn.conv3x3_bwd_data(_t(dy, cuda), w_bwd, relu_mask=_t(mask, cuda), dbias=dbias)
            mean, _ = Kn.bn_finalize(stats, M, cout, 1e-3, 0.99)
        torch.cuda.synchronize()
        outs[mode] = (y.cpu().numpy(), dx.cpu().numpy(), mean.cpu().numpy())
        dxm_ref = dx_ref * (mask > 0)
        assert float(np.linalg.norm(dxm.cpu().numpy() - dxm_ref) / np.linalg.norm(dxm_ref)) < 2e-6
        # column sums with cancellation: bounded by fp32 products over the column's absolute sum
        np.testing.assert_allclose(dbias.cpu().numpy(), 0.25 + dxm_ref.reshape(-1, cin).sum(0), rtol=0,
                                   atol=1e-6 * np.abs(dxm_ref).reshape(-1, cin).sum(0).max())
        rel = lambda a, r: float(np.linalg.norm(a - r) / np.linalg.norm(r))   # noqa: E731
        print(f"mode {mode}: fwd {rel(outs[mode][0], z):.3e} dgrad {rel(outs[mode][1], dx_ref):.3e}")
        assert rel(outs[mode][0], z) < 2e-6, (mode, rel(outs[mode][0], z))   # exact fp32 products
        assert rel(outs[mode][1], dx_ref) < 2e-6, (mode, rel(outs[mode][1], dx_ref))
        np.testing.assert_allclose(outs[mode][2], z.reshape(-1, cout).mean(0), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(outs[1][0], outs[0][0], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(outs[2][0], outs[1][0], rtol=1e-5, atol=1e-5)


# W = 11 / 37: one / several 8-window column segments of the window-centric
# routing pass, an odd width leaves an uncovered column for the 2x2/[2,2]
# pool, H = 7 an uncovered row for the 2-row pools.
@pytest.mark.parametrize("W", [11, 37])
@pytest.mark.parametrize("pool", [(2, 2, 2, 2), (2, 2, 2, 1), (3, 1, 3, 1)])
def test_bn_relu_pool(cuda, pool, W):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(sum(pool) + W)
    B, H, C = 2, 7 if pool[0] == 2 else 3, 32
    z = rng.standard_normal((B, H, W, C)).astype(np.float32)
    gamma = rng.standard_normal(C).astype(np.float32)
    beta = rng.standard_normal(C).astype(np.float32)
    a, mean, var, var_u, cache = G.bn_train(z, gamma, beta)
    y = G.relu(a)
    p_ref = G.maxpool(y, *pool)
    mean_d = _t(mean, cuda)
    inv_d = _t((1 / np.sqrt(var.astype(np.float64) + 1e-3)).astype(np.float32), cuda)
    tm = pool == (3, 1, 3, 1)
    p = Kn.bn_relu_pool_fwd(_t(z, cuda), mean_d, inv_d, _t(gamma, cuda), _t(beta, cuda), pool, time_major=tm)
    p = p.cpu().numpy()
    if tm:
        p = p.transpose(1, 0, 2)[:, None]
    np.testing.assert_allclose(p, p_ref, rtol=1e-5, atol=1e-5)
    dp = rng.standard_normal(p_ref.shape).astype(np.float32)
    dy = G.maxpool_bwd(y, dp, *pool)
    dz_ref, dg_ref, db_ref = G.bn_bwd(G.relu_bwd(y, dy), cache, gamma)
    dg = torch.zeros(C, device=cuda)
    db = torch.zeros(C, device=cuda)
    dp_d = _t(dp[:, 0].transpose(1, 0, 2) if tm else dp, cuda)
    dbias = torch.full((C,), 7.0, device=cuda)
    dz = Kn.bn_relu_pool_bwd(_t(z, cuda), dp_d, mean_d, inv_d, _t(gamma, cuda), _t(beta, cuda), pool, tm, dg, db,
                             accumulate=False, dbias=dbias)
    np.testing.assert_allclose(dz.cpu().numpy(), dz_ref, rtol=1e-4, atol=1e-5)
    # fused conv-bias gradient = column sums of dz (~0 up to rounding: BN removes the mean)
    np.testing.assert_allclose(dbias.cpu().numpy(), dz_ref.sum(axis=(0, 1, 2)), rtol=0, atol=1e-4)
    np.testing.assert_allclose(dg.cpu().numpy(), dg_ref, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(db.cpu().numpy(), db_ref, rtol=1e-4, atol=1e-5)


# The *_slab entry points (bias reduction left to the caller, e.g. on the side
# stream) give the same dx / dz and, after ocrk_slab_sum, the same dbias bits
# as the fused entry points; bf16 at a conv-tower shape (direct and GEMM routes).
@pytest.mark.parametrize("cin,cout,H,W", [(32, 32, 30, 60), (64, 128, 7, 126), (128, 256, 3, 125)])
def test_deferred_bias_reductions_match(cuda, cin, cout, H, W):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    g = torch.Generator(device=cuda).manual_seed(cin + cout)
    B = 8
    dy = torch.randn(B, H, W, cout, device=cuda, generator=g).bfloat16()
    w_bwd = (torch.randn(cin, 9 * cout, device=cuda, generator=g) / 30).bfloat16()
    mask = torch.randn(B, H, W, cin, device=cuda, generator=g).bfloat16()
    d1 = torch.full((cin,), 0.5, device=cuda)
    d2 = d1.clone()
    dx1 = Kn.conv3x3_bwd_data(dy, w_bwd, relu_mask=mask, dbias=d1)
    late = []
    dx2 = Kn.conv3x3_bwd_data(dy, w_bwd, relu_mask=mask, dbias=d2, defer=late)
    assert len(late) == 1 and torch.equal(d2, torch.full_like(d2, 0.5))
    late.pop()[0]()
    assert torch.equal(dx1, dx2) and torch.equal(d1, d2)
    for pool in [(2, 2, 2, 2), (2, 2, 2, 1), (3, 1, 3, 1)]:
        Hz = 3 if pool[0] == 3 else H
        z = torch.randn(B, Hz, W, cin, device=cuda, generator=g).bfloat16()
        kh, kw, sh, sw = pool
        tm = pool == (3, 1, 3, 1)
        Ho, Wo = (Hz - kh) // sh + 1, (W - kw) // sw + 1
        dp = torch.randn(*((Wo, B, cin) if tm else (B, Ho, Wo, cin)), device=cuda, generator=g).bfloat16()
        mean = torch.randn(cin, device=cuda, generator=g) * 0.1
        inv = torch.rand(cin, device=cuda, generator=g) + 0.5
        gamma = torch.randn(cin, device=cuda, generator=g)
        beta = torch.randn(cin, device=cuda, generator=g)
        outs = []
        for defer in (None, []):
            dg, db, dbias = torch.zeros(cin, device=cuda), torch.zeros(cin, device=cuda), torch.ones(cin, device=cuda)
            dz = Kn.bn_relu_pool_bwd(z, dp, mean, inv, gamma, beta, pool, tm, dg, db, dbias=dbias, defer=defer)
            if defer is not None:
                assert len(defer) == 1
                defer.pop()[0]()
            outs.append((dz, dg, db, dbias))
        for u, v in zip(*outs):
            assert torch.equal(u, v), pool


def test_slab_sum_matches_colsum_order(cuda):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    x = torch.randn(8, 4096, device=cuda)
    out = torch.full((4096,), 2.0, device=cuda)
    Kn.slab_sum(x, 8, 4096, 4096, out)
    np.testing.assert_allclose(out.cpu().numpy(), x.double().sum(0).cpu().numpy() + 2.0, rtol=0, atol=1e-5)
    strided = torch.randn(100, 96, device=cuda)
    out2 = torch.zeros(40, device=cuda)
    Kn.slab_sum(strided, 100, 40, 96, out2, accumulate=False)
    np.testing.assert_allclose(out2.cpu().numpy(), strided[:, :40].double().sum(0).cpu().numpy(), rtol=0, atol=1e-5)


@pytest.mark.parametrize("nslab,nc", [(2085, 512), (777, 64), (2048, 256), (31, 128)])
def test_slab_sum_fixed_order_bits(cuda, nslab, nc):
    """The one-launch form's order (tensor_ops.hip slab_sum_fused): row group rg
    of 16 adds rows rg, rg + 16, ... in sequence (double), then the 16 groups in
    order; the 32- / 8- / 1-row load batches must not change it."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    g = torch.Generator(device="cpu").manual_seed(nslab)
    x = torch.randn(nslab, nc, generator=g) * torch.rand(nslab, 1, generator=g) * 10
    out = torch.zeros(nc, device=cuda)
    Kn.slab_sum(x.to(cuda), nslab, nc, nc, out, accumulate=False)
    xd = x.double().numpy()
    groups = [np.cumsum(xd[rg::16], axis=0)[-1] if rg < nslab else np.zeros(nc) for rg in range(16)]
    want = np.cumsum(np.stack(groups), axis=0)[-1].astype(np.float32)
    np.testing.assert_array_equal(out.cpu().numpy(), want)


# column sums (bias gradients of the odd convs, recurrent and logits layers)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N", [(37, 64), (5000, 24), (3001, 4096), (20000, 256)])
def test_colsum(cuda, dtype, M, N):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(M + N)
    x = rng.standard_normal((M, N)).astype(np.float32)
    xd = _t(x, cuda, dtype)
    ref = xd.double().sum(0).cpu().numpy() + 1.5
    out = torch.full((N,), 1.5, device=cuda)
    Kn.colsum(xd, M, N, out, accumulate=True)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=0, atol=1e-5 * np.sqrt(M) + 1e-5)
    out2 = torch.full((N,), 9.0, device=cuda)
    Kn.colsum(xd, M, N, out2, accumulate=False)
    np.testing.assert_allclose(out2.cpu().numpy(), ref - 1.5, rtol=0, atol=1e-5 * np.sqrt(M) + 1e-5)


# --------------------------------------------------------------------- LSTM
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_lstm_layer_fwd_bwd(cuda, dtype):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(5)
    T, B, n_in, H = 9, 64, 64, 256
    x = rng.standard_normal((T, B, n_in)).astype(np.float32)
    seq = rng.integers(1, T + 1, B).astype(np.int32)
    seq[0] = T
    ks = [(rng.standard_normal((n_in + H, 4 * H)) * 0.2).astype(np.float32) for _ in range(2)]
    bs = [(rng.standard_normal(4 * H) * 0.2).astype(np.float32) for _ in range(2)]
    if dtype == torch.bfloat16:
        x = torch.from_numpy(x).bfloat16().float().numpy()
        ks = [torch.from_numpy(k).bfloat16().float().numpy() for k in ks]
    outs, caches = [], []
    for d, rev in enumerate((False, True)):
        o, c = G.lstm_dir_fwd(x, seq, ks[d], bs[d], rev)
        outs.append(o)
        caches.append(c)
    ref = np.concatenate(outs, axis=2)
    # device images, as ParamStore.lstm_images builds them
    G4 = 4 * H
    wxT = np.concatenate([k[:n_in].T for k in ks], 0)              # [8H][In]
    wx = np.concatenate([k[:n_in] for k in ks], 1)                 # [In][8H]
    whT = np.stack([k[n_in:].T for k in ks])                       # [2][4H][H]
    wh = np.stack([k[n_in:] for k in ks])                          # [2][H][4H]
    bias = np.concatenate(bs)
    seq_d = _t(seq, cuda)
    gx = Kn.gemm(_t(x.reshape(T * B, n_in), cuda, dtype), _t(wxT, cuda, dtype), trans_b=True, bias=_t(bias, cuda),
                 out_dtype=dtype)
    out, hprev, cprev, acts = Kn.lstm_fwd(gx, _t(whT, cuda, dtype), seq_d, T, B, H, dtype)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    assert _rel(out.float().cpu().numpy(), ref) < tol
    dout = rng.standard_normal(ref.shape).astype(np.float32)
    if dtype == torch.bfloat16:
        dout = torch.from_numpy(dout).bfloat16().float().numpy()
    dG = Kn.lstm_bwd(_t(wh, cuda, dtype), seq_d, _t(dout, cuda, dtype), cprev, acts, T, B, H)
    dx_dev = Kn.gemm(dG.view(T * B, 2 * G4), _t(wx, cuda, dtype), trans_b=True).view(T, B, n_in)
    dxr = np.zeros_like(x)
    for d in range(2):
        ddx, dk, db = G.lstm_dir_bwd(np.ascontiguousarray(dout[:, :, d * H:(d + 1) * H]), caches[d], ks[d], n_in)
        dxr += ddx
        dgd = dG.view(T * B, 2 * G4)[:, d * G4:]
        gk = torch.zeros(n_in + H, G4, device=cuda)
        Kn.gemm(_t(x, cuda, dtype), dgd, trans_a=True, out=gk, accumulate=True, M=n_in, N=G4, K=T * B, lda=n_in,
                ldb=2 * G4, ldc=G4)
        Kn.gemm(hprev.view(T * B, 2 * H)[:, d * H:], dgd, trans_a=True, out=gk[n_in:], accumulate=True, M=H, N=G4,
                K=T * B, lda=2 * H, ldb=2 * G4, ldc=G4, splits=2)
        assert _rel(gk.cpu().numpy(), dk) < (1e-4 if dtype == torch.float32 else 5e-2)
    assert _rel(dx_dev.cpu().numpy(), dxr) < (1e-4 if dtype == torch.float32 else 5e-2)


def test_adam_matches_oracle(cuda):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(2)
    n = 1000
    p, g = rng.standard_normal(n).astype(np.float32), rng.standard_normal(n).astype(np.float32)
    m, v = np.zeros(n, np.float32), np.zeros(n, np.float32)
    pd, gd, md, vd = _t(p, cuda), _t(g, cuda), _t(m, cuda), _t(v, cuda)
    for t in (1, 2, 3):
        lr = G.learning_rate(t - 1)
        p, m, v = G.adam_update(p, g, m, v, lr, t)
        lr_t = lr * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        Kn.adam_(pd, gd, md, vd, lr_t)
    np.testing.assert_allclose(pd.cpu().numpy(), p, rtol=1e-6, atol=1e-7)
    # the device forms (1 - beta2) in float32 like TF's ApplyAdam (0.00099998713 vs 0.001)
    np.testing.assert_allclose(vd.cpu().numpy(), v, rtol=3e-5, atol=1e-9)


def test_adam_zero_grad_form(cuda):
    """ocrk_adam_ex with OCRK_ADAM_ZERO_GRAD (the Trainer's update): the same
    bits as the plain update, and the gradient cleared as it is read (a length
    that is not a multiple of 4 exercises the scalar tail)."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(3)
    n = 1003
    p, g = rng.standard_normal(n).astype(np.float32), rng.standard_normal(n).astype(np.float32)
    a = [_t(x, cuda) for x in (p, g, np.zeros(n, np.float32), np.zeros(n, np.float32))]
    b = [_t(x, cuda) for x in (p, g, np.zeros(n, np.float32), np.zeros(n, np.float32))]
    Kn.adam_(*a, 1e-3, grad_scale=0.5)
    Kn.adam_(*b, 1e-3, grad_scale=0.5, zero_grad=True)
    for x, y in zip((a[0], a[2], a[3]), (b[0], b[2], b[3])):
        assert torch.equal(x, y)
    assert torch.equal(a[1], _t(g, cuda)) and torch.count_nonzero(b[1]).item() == 0


def test_gemm_weight_grad_form_bf16(cuda):
    """dW += x^T . dG as the recurrent backward issues it (bf16 operands, f32
    accumulate into an existing gradient, dG a strided column view, split-K
    requested): the split-K TN engine must give the float64 product."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(5)
    R, n_in, G4 = 1000, 96, 256
    x = torch.from_numpy(rng.standard_normal((R, n_in)).astype(np.float32)).bfloat16()
    dG = torch.from_numpy(rng.standard_normal((R, 2 * G4)).astype(np.float32)).bfloat16()
    C0 = rng.standard_normal((n_in, G4)).astype(np.float32)
    out = _t(C0, cuda)
    xd, dGd = x.to(cuda), dG.to(cuda)
    Kn.gemm(xd, dGd[:, G4:], trans_a=True, out=out, accumulate=True, M=n_in, N=G4, K=R, lda=n_in, ldb=2 * G4,
            ldc=G4, splits=4)
    ref = C0 + x.float().numpy().astype(np.float64).T @ dG.float().numpy()[:, G4:].astype(np.float64)
    assert _rel(out.cpu().numpy(), ref) < 1e-5


# the weight gradients by image rows (conv_rows.hip) against the chunked direct /
# TN engines (OCRK_CONV_ROWS=0) and a float64 reference: conv2 at the bench's 30 x 254
# rows, conv3 / conv4, and conv5 / conv6 as 64 x 64 channel blocks (2 / 4 blocks)
@pytest.mark.parametrize("B,H,W,C,CO", [(6, 30, 254, 32, 32), (5, 15, 127, 32, 64), (5, 15, 127, 64, 64),
                                        (3, 4, 9, 64, 64), (3, 7, 126, 64, 128), (3, 7, 126, 128, 128),
                                        (2, 3, 9, 128, 128), (3, 3, 125, 128, 256), (2, 3, 125, 256, 256)])
def test_conv2_wgrad_rows_matches(cuda, ocrk_opts, B, H, W, C, CO):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    g = torch.Generator(device=cuda).manual_seed(5)
    x = torch.randn(B, H, W, C, device=cuda, generator=g).bfloat16()
    dy = torch.randn(B, H, W, CO, device=cuda, generator=g).bfloat16()
    ref = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2).transpose(0, 1),
                                     dy.double().permute(0, 3, 1, 2).transpose(0, 1), padding=1)  # [ci][co][3][3]
    ref = ref.permute(2, 3, 0, 1).contiguous()                                                # HWIO
    outs = []
    ocrk_opts("CONV_WGRAD_BLOCKS", 2)           # conv7 / conv8 blocks too (opt-in)
    for mode in ("1", "0"):
        ocrk_opts("CONV_ROWS", int(mode))
        dw = torch.full((3, 3, C, CO), 0.5, device=cuda)
        Kn.conv3x3_bwd_weight(x, dy, dw, accumulate=True)
        outs.append(dw.double() - 0.5)
    for o in outs:
        torch.testing.assert_close(o, ref, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-5, atol=1e-3)


# conv2's data gradient by image rows (conv_rows.hip) against the chunked direct
# kernel (same bits: same products, same k order per output) and float64
def test_conv2_dgrad_rows_matches(cuda, ocrk_opts):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    g = torch.Generator(device=cuda).manual_seed(7)
    for B, H, W in [(4, 30, 254), (3, 7, 37), (2, 1, 5)]:
        C = 32
        dy = torch.randn(B, H, W, C, device=cuda, generator=g).bfloat16()
        w = (torch.randn(3, 3, C, C, device=cuda, generator=g) / 17).bfloat16()          # HWIO
        w_bwd = w.permute(2, 0, 1, 3).contiguous().view(C, 9 * C)                          # [ci][kh][kw][co]
        mask = torch.randn(B, H, W, C, device=cuda, generator=g).bfloat16()
        ref = torch.nn.functional.conv_transpose2d(dy.double().permute(0, 3, 1, 2),
                                                   w.double().permute(2, 3, 0, 1).transpose(0, 1), padding=1)
        ref = ref.permute(0, 2, 3, 1) * (mask.double() > 0)
        outs = []
        for mode in ("1", "0"):
            ocrk_opts("CONV_ROWS", int(mode))
            outs.append(Kn.conv3x3_bwd_data(dy, w_bwd, relu_mask=mask))
        torch.testing.assert_close(outs[0].double(), ref, rtol=2e-2, atol=2e-2)
        assert torch.equal(outs[0], outs[1]), (B, H, W)


# conv2's forward by image rows: the same z bits as the chunked direct kernel,
# BatchNorm mean / invstd from the per-row partials within float tolerance
@pytest.mark.parametrize("CI,CO,shapes", [(32, 32, [(4, 30, 254), (3, 7, 37), (2, 1, 5)]),
                                          (32, 64, [(4, 15, 127), (2, 3, 20)]),
                                          (64, 64, [(4, 15, 127), (2, 2, 9)]),
                                          (64, 128, [(4, 7, 126), (2, 5, 17)])])
def test_conv2_fwd_rowstats_matches(cuda, ocrk_opts, CI, CO, shapes):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    g = torch.Generator(device=cuda).manual_seed(9)
    for B, H, W in shapes:
        C = CO
        x = torch.randn(B, H, W, CI, device=cuda, generator=g).bfloat16()
        w_nk = (torch.randn(C, 9 * CI, device=cuda, generator=g) / 17).bfloat16()
        bias = torch.randn(C, device=cuda, generator=g)
        assert Kn.conv3x3_fwd_rowstats_ok(x, C)
        z, st = Kn.conv3x3_fwd_rowstats(x, w_nk, bias)
        M = B * H * W
        ocrk_opts("CONV_ROWS", 0)
        st_ref = torch.empty(Kn.conv_stats_tiles(M), 2, C, device=cuda)
        z_ref = Kn.conv3x3_fwd(x, w_nk, bias, relu=False, stats=st_ref)
        ocrk_opts.reset("CONV_ROWS")
        assert torch.equal(z, z_ref), (B, H, W)
        m1, i1 = Kn.bn_finalize(st, M, C, 1e-3, 0.99, tile_rows=W)
        m2, i2 = Kn.bn_finalize(st_ref, M, C, 1e-3, 0.99)
        zf = z.double().view(-1, C)
        # the partials are of the f32 values before the bf16 rounding of z: against z
        # only to bf16 rounding (the tight check is the 128-tile path below)
        tol = 8e-3 * float(zf.abs().max())
        torch.testing.assert_close(m1.double(), zf.mean(0), rtol=0, atol=tol)
        torch.testing.assert_close(i1.double(), 1 / torch.sqrt(zf.var(0, unbiased=False) + 1e-3), rtol=2e-2, atol=0)
        torch.testing.assert_close(m1, m2, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(i1, i2, rtol=1e-5, atol=1e-6)
        # no-statistics forward (serving) takes the row kernel too: same bits
        assert torch.equal(Kn.conv3x3_fwd(x, w_nk, bias, relu=True), torch.relu(z_ref.float()).bfloat16())


# the wider layers' data gradient by rows (conv4: 64 <- 64 with the ReLU mask and
# the producer's bias sums, conv5: 64 <- 128 plain) against the GEMM path
@pytest.mark.parametrize("CI,CO,H,W,masked", [(64, 64, 15, 127, True), (64, 64, 15, 127, False),
                                              (64, 64, 3, 20, True)])
def test_dgrad_rows_wide_matches(cuda, ocrk_opts, CI, CO, H, W, masked):
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    g = torch.Generator(device=cuda).manual_seed(CI + CO + W)
    B = 5
    dy = torch.randn(B, H, W, CO, device=cuda, generator=g).bfloat16()
    w_bwd = (torch.randn(CI, 9 * CO, device=cuda, generator=g) / 20).bfloat16()
    mask = torch.randn(B, H, W, CI, device=cuda, generator=g).bfloat16() if masked else None
    outs = []
    ocrk_opts("CONV_WGRAD_BLOCKS", 2)           # conv7 / conv8 blocks too (opt-in)
    for mode in ("1", "0"):
        ocrk_opts("CONV_ROWS", int(mode))
        db = torch.full((CI,), 0.25, device=cuda) if masked else None
        dx = Kn.conv3x3_bwd_data(dy, w_bwd, relu_mask=mask, dbias=db)
        outs.append((dx, db))
    assert torch.equal(outs[0][0], outs[1][0])
    if masked:
        torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-3)
        # against the bf16-rounded dx only to rounding noise (the sums are of the f32 values)
        ref = outs[1][0].double().view(-1, CI).sum(0) + 0.25
        n = outs[1][0].numel() // CI
        torch.testing.assert_close(outs[0][1].double(), ref, rtol=0, atol=0.01 * n ** 0.5)
