"""bf16 parity of the BENCHED routes against the float64 oracle.

The headline bench runs bf16 (BASELINE.json configs[2]); these tests pin the
bf16 engines it uses at the layer shapes it uses, against the oracle on the
SAME bf16-rounded operands (so the only differences are the kernels' fp32
accumulation order and the bf16 rounding of their outputs):
  * the NT im2col conv engine (forward with the BN-statistics epilogue and the
    ReLU epilogue, backward-data with the producer's ReLU mask and the fused
    bias gradient) and the TN weight-gradient engine, at conv2 (32->32,
    30x254) and conv8 (256->256, 3x125) -- model.py:84-109,126-146;
  * the ping-pong GEMM engine (gemm_pp) with a bias epilogue and bf16 C on the
    recurrent input-projection and data-gradient shapes -- model_bu.py:186-192;
  * the whole bf16 train step (persistent LSTM, every default route) at the
    bench's width and LSTM sizes, B=64 (T*B=8000 rows: the same kernels and
    tile configurations as B=256; two float64 oracle runs of a 256-crop step
    take minutes of host time), loss / logits / every variable's gradient,
    with the bf16 bounds stated in the test.
"""
import numpy as np
import pytest
import torch

from oracle import ref_graph as G
from oracle import ref_model as M

pytestmark = pytest.mark.gpu


def _bf(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).bfloat16().float().numpy()


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


# bf16 output rounding alone is 2^-9 relative per element (~1.6e-3 RMS on
# random data); accumulation-order differences are below 1e-5
BF16_OUT = 4e-3


@pytest.mark.parametrize("B,H,W,cin,cout", [(4, 30, 254, 32, 32), (4, 15, 127, 32, 64), (4, 15, 127, 64, 64),
                                             (4, 7, 126, 64, 128), (8, 3, 125, 128, 256), (16, 3, 125, 256, 256)])
@pytest.mark.parametrize("direct", ["1", "2"])
def test_bf16_conv_engines_at_layer_shapes(cuda, ocrk_opts, B, H, W, cin, cout, direct):
    """conv2..conv5 shapes run the direct kernel (conv_direct.hip) forward and
    backward-data where it is routed (OCRK_CONV_DIRECT=1, the default: Cin 32
    or dgrad output 32) or wherever it covers the shape (=2), conv8 the
    implicit GEMM; ragged tails (B*H*W not a multiple of the 128-pixel tile)."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    ocrk_opts("CONV_DIRECT", int(direct))
    rng = np.random.default_rng(cin * 7 + W)
    x = _bf(rng.standard_normal((B, H, W, cin)))
    w = _bf(rng.standard_normal((3, 3, cin, cout)) / np.sqrt(9 * cin))
    b = rng.standard_normal(cout).astype(np.float32)
    x64, w64 = x.astype(np.float64), w.astype(np.float64)
    z = G.conv2d(x64, w64, b.astype(np.float64), "same")
    xd = torch.from_numpy(x).to(cuda).bfloat16()
    wd = torch.from_numpy(w).to(cuda)
    w_nk = Kn.permute3(wd, 9 * cin, cout, 1, torch.bfloat16).view(cout, 9 * cin)
    w_bwd = Kn.permute3(wd, 9, cin, cout, torch.bfloat16).view(cin, 9 * cout)
    M_ = B * H * W
    # forward with the BN statistics epilogue (conv2/4/6/8) and with ReLU (conv3/5/7)
    stats = torch.empty(Kn.conv_stats_tiles(M_), 2, cout, device=cuda)
    y = Kn.conv3x3_fwd(xd, w_nk, torch.from_numpy(b).to(cuda), False, stats=stats)
    assert _rel(y.float().cpu().numpy(), z) < BF16_OUT
    mean, invstd = Kn.bn_finalize(stats, M_, cout, 1e-3, 0.99)
    zf = z.reshape(-1, cout)
    np.testing.assert_allclose(mean.cpu().numpy(), zf.mean(0), rtol=1e-4, atol=1e-4 * np.abs(zf).max())
    np.testing.assert_allclose(invstd.cpu().numpy(), 1 / np.sqrt(zf.var(0) + 1e-3), rtol=1e-3)
    yr = Kn.conv3x3_fwd(xd, w_nk, torch.from_numpy(b).to(cuda), True)
    assert _rel(yr.float().cpu().numpy(), np.maximum(z, 0)) < BF16_OUT
    # backward-data with the producer's ReLU mask and the fused bias gradient
    dy = _bf(rng.standard_normal(z.shape))
    dx_ref, dw_ref, _ = G.conv2d_bwd(x64, w64, dy.astype(np.float64), "same")
    mask = _bf(rng.standard_normal(x.shape))
    dmask = dx_ref * (mask > 0)
    dbias = torch.zeros(cin, device=cuda)
    dx = Kn.conv3x3_bwd_data(torch.from_numpy(dy).to(cuda).bfloat16(), w_bwd,
                             relu_mask=torch.from_numpy(mask).to(cuda).bfloat16(), dbias=dbias)
    assert _rel(dx.float().cpu().numpy(), dmask) < BF16_OUT
    # the bias gradient sums the fp32 values before their bf16 rounding
    assert _rel(dbias.cpu().numpy(), dmask.reshape(-1, cin).sum(0)) < 1e-4
    # backward-data without mask / bias gradient (the odd layers' dx)
    dx_plain = Kn.conv3x3_bwd_data(torch.from_numpy(dy).to(cuda).bfloat16(), w_bwd)
    assert _rel(dx_plain.float().cpu().numpy(), dx_ref) < BF16_OUT
    # TN weight gradient, f32 accumulation over B*H*W pixels (Cin % 64 == 0 and
    # 9 Cin, Cout >= 256: the 256 x 256 ping-pong engine's im2col mode)
    dw = torch.zeros(3, 3, cin, cout, device=cuda)
    Kn.conv3x3_bwd_weight(xd, torch.from_numpy(dy).to(cuda).bfloat16(), dw, accumulate=False)
    assert _rel(dw.cpu().numpy(), dw_ref) < 1e-4


def _relu_bits(y):
    """conv1's ReLU bit mask on the host: u8 [..., C/8], bit c of byte g = y[..., 8 g + c] > 0."""
    pos = (np.asarray(y) > 0).reshape(*y.shape[:-1], y.shape[-1] // 8, 8).astype(np.uint8)
    return (pos << np.arange(8, dtype=np.uint8)).sum(-1).astype(np.uint8)


@pytest.mark.parametrize("x_u8", [True, False])
def test_conv1_fwd_relu_bits(cuda, x_u8):
    """ocrk_conv1_fwd_relu_bits: the same y bits as ocrk_conv1_fwd, and the bit
    mask of y > 0 (the fused conv2 backward's ReLU mask)."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(5 + x_u8)
    img = rng.integers(0, 256, (3, 32, 131)).astype(np.uint8)
    x = torch.from_numpy(img).to(cuda) if x_u8 else Kn.preprocess(torch.from_numpy(img).to(cuda), torch.bfloat16)
    w = torch.from_numpy(rng.standard_normal((3, 3, 1, 32)).astype(np.float32)).to(cuda)
    b = torch.from_numpy(rng.standard_normal(32).astype(np.float32) * 0.1).to(cuda)
    y = Kn.conv1_fwd(x, w, b, torch.bfloat16)
    y2, bits = Kn.conv1_fwd(x, w, b, torch.bfloat16, relu_bits=True)
    assert torch.equal(y, y2)
    assert bits.shape == (3, 30, 129, 4)
    np.testing.assert_array_equal(bits.cpu().numpy(), _relu_bits(y.float().cpu().numpy()))


@pytest.mark.parametrize("B,IH,IW", [(4, 32, 256), (3, 17, 130), (2, 3, 9), (5, 32, 70)])
@pytest.mark.parametrize("x_u8", [True, False])
def test_conv12_fused_forward(cuda, B, IH, IW, x_u8):
    """conv1 -> conv2 in one row walk (ocrk_conv12_fwd, the bench's first block): y1 (conv1
    on the MFMA, hi + lo operands) against the float64 conv1 and the fp32 VALU conv1 kernel
    (bf16 rounding level); its bit mask = y1 > 0; z and the per-row BN partials bit-identical
    to the conv2 row kernel run on the same y1 (the same MFMA sequence)."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(IH * 100 + IW + 7 * x_u8)
    img = rng.integers(0, 256, (B, IH, IW)).astype(np.uint8)
    w1 = rng.standard_normal((3, 3, 1, 32)).astype(np.float32)
    b1 = (rng.standard_normal(32) * 0.3).astype(np.float32)
    w2 = _bf(rng.standard_normal((3, 3, 32, 32)) / np.sqrt(288))
    b2 = rng.standard_normal(32).astype(np.float32)
    if x_u8:
        xd = torch.from_numpy(img).to(cuda)
        x64 = G.preprocess(img).astype(np.float64)
    else:
        xf = _bf(rng.standard_normal((B, IH, IW)))
        xd = torch.from_numpy(xf).to(cuda).bfloat16()
        x64 = xf.astype(np.float64)
    w1d, b1d = torch.from_numpy(w1).to(cuda), torch.from_numpy(b1).to(cuda)
    w_nk = Kn.permute3(torch.from_numpy(w2).to(cuda), 9 * 32, 32, 1, torch.bfloat16).view(32, 9 * 32)
    b2d = torch.from_numpy(b2).to(cuda)
    assert Kn.conv12_fwd_ok(xd, torch.bfloat16)
    y1, bits, z, stats = Kn.conv12_fwd(xd, w1d, b1d, w_nk, b2d)
    y1_ref = G.relu(G.conv2d(x64[..., None], w1.astype(np.float64), b1.astype(np.float64), "valid"))
    y1f = y1.float().cpu().numpy()
    assert _rel(y1f, y1_ref) < BF16_OUT
    y1_valu = Kn.conv1_fwd(xd, w1d, b1d, torch.bfloat16).float().cpu().numpy()
    differ = np.abs(y1f - y1_valu) > 2 ** -7 * np.abs(y1_valu) + 1e-6
    assert differ.mean() < 1e-3, differ.mean()              # at most a last-bit rounding apart
    np.testing.assert_array_equal(bits.cpu().numpy(), _relu_bits(y1f))
    z2, st2 = Kn.conv3x3_fwd_rowstats(y1, w_nk, b2d)
    torch.cuda.synchronize()
    assert torch.equal(z, z2)
    assert torch.equal(stats, st2)
    # without y1 (the fused backward, ocrk_conv12_bwd, recomputes it): the same bits, z and partials
    none, bits3, z3, st3 = Kn.conv12_fwd(xd, w1d, b1d, w_nk, b2d, want_y1=False)
    torch.cuda.synchronize()
    assert none is None
    assert torch.equal(bits, bits3) and torch.equal(z, z3) and torch.equal(stats, st3)


@pytest.mark.parametrize("B,H,W,cin,cout,cnext", [(4, 15, 127, 32, 64, 64), (4, 7, 126, 64, 128, 128),
                                                  (8, 3, 125, 128, 256, 256), (3, 5, 37, 64, 64, 64)])
def test_relu_bit_masks_conv_pair(cuda, B, H, W, cin, cout, cnext):
    """conv_{odd}'s forward with its ReLU bit mask (ocrk_conv3x3_fwd_relu_bits: the wide row
    kernels for conv3 / conv5, the NT engine's staged epilogue for conv7) gives the same y
    bits as the plain forward and the bits of y > 0; conv_{even}'s backward-data with that
    bit mask (ocrk_conv3x3_bwd_data_bits: rows kernel for conv4, NT for conv6 / conv8) the
    same dx and producer bias gradient as with the bf16 y as the mask."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(cin + cout + W)
    x = torch.from_numpy(_bf(rng.standard_normal((B, H, W, cin)))).to(cuda).bfloat16()
    w = torch.from_numpy(_bf(rng.standard_normal((3, 3, cin, cout)) / np.sqrt(9 * cin))).to(cuda)
    b = torch.from_numpy(rng.standard_normal(cout).astype(np.float32) * 0.3).to(cuda)
    w_nk = Kn.permute3(w, 9 * cin, cout, 1, torch.bfloat16).view(cout, 9 * cin)
    assert Kn.relu_bits_ok((B, H, W), cin, cout, cnext, torch.bfloat16)
    y = Kn.conv3x3_fwd(x, w_nk, b, True)
    y2, bits = Kn.conv3x3_fwd_relu_bits(x, w_nk, b)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    np.testing.assert_array_equal(bits.cpu().numpy(), _relu_bits(y.float().cpu().numpy()))
    w2 = torch.from_numpy(_bf(rng.standard_normal((3, 3, cout, cnext)) / np.sqrt(9 * cout))).to(cuda)
    w_bwd = Kn.permute3(w2, 9, cout, cnext, torch.bfloat16).view(cout, 9 * cnext)
    dz = torch.from_numpy(_bf(rng.standard_normal((B, H, W, cnext)))).to(cuda).bfloat16()
    db1, db2 = torch.zeros(cout, device=cuda), torch.zeros(cout, device=cuda)
    dx1 = Kn.conv3x3_bwd_data(dz, w_bwd, relu_mask=y, dbias=db1)
    dx2 = Kn.conv3x3_bwd_data(dz, w_bwd, dbias=db2, relu_bits=bits)
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx2)
    assert torch.equal(db1, db2)


@pytest.mark.parametrize("B,IH,IW", [(4, 32, 256), (3, 17, 130), (2, 3, 9), (5, 32, 70)])
@pytest.mark.parametrize("x_u8", [True, False])
@pytest.mark.parametrize("mask", ["bf16", "bits"])
def test_conv2_bwd_data_fused_conv1_wgrad(cuda, B, IH, IW, x_u8, mask):
    """conv2's backward-data with conv1's weight gradient contracted in
    (ocrk_conv2_bwd_data_conv1_wgrad, the bench's k = 1 backward): against the
    float64 oracle on the kernel's own bf16 dy1 (relu'(y1) . conv2^T dz, rounded
    once), and against the unfused pair (bf16 dy1 stored, then conv1_bwd_weight).
    Shapes: the bench crop (30 x 254), odd band heights (15 rows: 8 + 7), one
    conv1 output row (the second band empty: a zero partial), a narrow row."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(IH * 1000 + IW + x_u8)
    H, W = IH - 2, IW - 2
    img = rng.integers(0, 256, (B, IH, IW)).astype(np.uint8)
    x = G.preprocess(img) if x_u8 else _bf(rng.standard_normal((B, IH, IW)))
    w1 = rng.standard_normal((3, 3, 1, 32)).astype(np.float32)
    w2 = _bf(rng.standard_normal((3, 3, 32, 32)) / np.sqrt(288))
    y1 = _bf(rng.standard_normal((B, H, W, 32)))                    # conv1's output: the ReLU mask
    dz = _bf(rng.standard_normal((B, H, W, 32)))
    dx_ref, _, _ = G.conv2d_bwd(y1.astype(np.float64), w2.astype(np.float64), dz.astype(np.float64), "same")
    dy1 = _bf(dx_ref * (y1 > 0))
    _, dw_ref, db_ref = G.conv2d_bwd(np.asarray(x, np.float64)[..., None], w1.astype(np.float64),
                                     dy1.astype(np.float64), "valid", need_dx=False)
    xd = torch.from_numpy(img).to(cuda) if x_u8 else torch.from_numpy(x).to(cuda).bfloat16()
    dzd = torch.from_numpy(dz).to(cuda).bfloat16()
    y1d = torch.from_numpy(y1).to(cuda).bfloat16()
    w_bwd = Kn.permute3(torch.from_numpy(w2).to(cuda), 9, 32, 32, torch.bfloat16).view(32, 9 * 32)
    assert Kn.conv2_bwd_data_conv1_wgrad_ok(dzd, xd)
    prev_w = rng.standard_normal((3, 3, 1, 32)).astype(np.float32)
    prev_b = rng.standard_normal(32).astype(np.float32)
    dw = torch.from_numpy(prev_w).to(cuda)
    db = torch.from_numpy(prev_b).to(cuda)
    if mask == "bits":
        bits = torch.from_numpy(_relu_bits(y1)).to(cuda)
        Kn.conv2_bwd_data_conv1_wgrad(dzd, w_bwd, None, xd, dw, db, accumulate=True, relu_bits=bits)
    else:
        Kn.conv2_bwd_data_conv1_wgrad(dzd, w_bwd, y1d, xd, dw, db, accumulate=True)
    # f32 accumulation over B*H*W pixels of bf16 dy1 x (hi + lo) x: ~1e-6 relative; the
    # reference's dy1 is the float64 sum rounded once, so the ~5e-5 of elements whose
    # fp32 sum rounds to the neighbouring bf16 value add up to ~2e-5 here
    assert _rel(dw.cpu().numpy() - prev_w, dw_ref) < 1e-4
    assert _rel(db.cpu().numpy() - prev_b, db_ref) < 1e-4
    # the unfused pair on the same bf16 dy1 bits (only the summation order and the
    # hi + lo split of x differ)
    dy1d = Kn.conv3x3_bwd_data(dzd, w_bwd, relu_mask=y1d)
    dw2, db2 = torch.zeros(3, 3, 1, 32, device=cuda), torch.zeros(32, device=cuda)
    Kn.conv1_bwd_weight(xd, dy1d, dw2, db2, accumulate=False)
    assert _rel(dw2.cpu().numpy(), dw_ref) < 1e-4
    assert _rel(dw.cpu().numpy() - prev_w, dw2.cpu().numpy()) < 2e-5
    assert _rel(db.cpu().numpy() - prev_b, db2.cpu().numpy()) < 2e-5
    np.testing.assert_allclose(dw.cpu().numpy() - prev_w, dw2.cpu().numpy(), rtol=1e-3,
                               atol=1e-5 * float(np.abs(dw_ref).max()))


@pytest.mark.parametrize("B,IH,IW", [(4, 32, 256), (3, 17, 130), (2, 3, 9), (5, 32, 70), (1, 32, 256)])
@pytest.mark.parametrize("x_u8", [True, False])
@pytest.mark.parametrize("mask", ["bf16", "bits"])
def test_conv12_bwd_fused(cuda, B, IH, IW, x_u8, mask):
    """conv1 -> conv2's whole backward as one row walk (ocrk_conv12_bwd, the bench's k = 1
    backward): conv2's weight gradient with y1 recomputed from the image against the
    float64 sum over the forward's y1 (ocrk_conv12_fwd) and against the separate weight
    gradient kernel on that y1 (summation order only); conv1's weight / bias gradients as
    ocrk_conv2_bwd_data_conv1_wgrad's. Shapes: the bench crop, odd heights, one conv1 output
    row, a narrow row, B = 1 (a single partial)."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(IH * 1000 + IW + x_u8 + 17 * B)
    H, W = IH - 2, IW - 2
    img = rng.integers(0, 256, (B, IH, IW)).astype(np.uint8)
    xf = _bf(rng.standard_normal((B, IH, IW)))
    xd = torch.from_numpy(img).to(cuda) if x_u8 else torch.from_numpy(xf).to(cuda).bfloat16()
    w1 = rng.standard_normal((3, 3, 1, 32)).astype(np.float32)
    b1 = (rng.standard_normal(32) * 0.3).astype(np.float32)
    w2 = _bf(rng.standard_normal((3, 3, 32, 32)) / np.sqrt(288))
    w1d, b1d = torch.from_numpy(w1).to(cuda), torch.from_numpy(b1).to(cuda)
    w_nk = Kn.permute3(torch.from_numpy(w2).to(cuda), 9 * 32, 32, 1, torch.bfloat16).view(32, 9 * 32)
    w_bwd = Kn.permute3(torch.from_numpy(w2).to(cuda), 9, 32, 32, torch.bfloat16).view(32, 9 * 32)
    y1d, bits, _, _ = Kn.conv12_fwd(xd, w1d, b1d, w_nk, torch.zeros(32, device=cuda))
    dz = _bf(rng.standard_normal((B, H, W, 32)))
    dzd = torch.from_numpy(dz).to(cuda).bfloat16()
    assert Kn.conv12_bwd_ok(xd, torch.bfloat16)
    prev = [rng.standard_normal(s).astype(np.float32) for s in ((3, 3, 32, 32), (3, 3, 1, 32), (32,))]
    dw2, dw1, db1 = (torch.from_numpy(p).to(cuda) for p in prev)
    if mask == "bits":
        Kn.conv12_bwd(dzd, w_bwd, xd, w1d, b1d, dw2, dw1, db1, relu_bits=bits)
    else:
        Kn.conv12_bwd(dzd, w_bwd, xd, w1d, b1d, dw2, dw1, db1, relu_mask=y1d)
    got2, got1, gotb = (t.cpu().numpy() - p for t, p in zip((dw2, dw1, db1), prev))
    y1 = y1d.float().cpu().numpy().astype(np.float64)
    _, dw2_ref, _ = G.conv2d_bwd(y1, w2.astype(np.float64), dz.astype(np.float64), "same", need_dx=False)
    assert _rel(got2, dw2_ref) < 1e-5
    # the separate weight-gradient kernel on the forward's y1: the same products, another order
    sep = torch.zeros(3, 3, 32, 32, device=cuda)
    Kn.conv3x3_bwd_weight(y1d, dzd, sep, accumulate=False)
    assert _rel(got2, sep.cpu().numpy()) < 1e-5
    # conv1's gradients: the two-output walk's (one band per image) against the data-gradient
    # walk's (two bands per image) -- the same dy1 bits, another partial grouping
    c1w, c1b = torch.zeros(3, 3, 1, 32, device=cuda), torch.zeros(32, device=cuda)
    if mask == "bits":
        Kn.conv2_bwd_data_conv1_wgrad(dzd, w_bwd, None, xd, c1w, c1b, accumulate=False, relu_bits=bits)
    else:
        Kn.conv2_bwd_data_conv1_wgrad(dzd, w_bwd, y1d, xd, c1w, c1b, accumulate=False)
    assert _rel(got1, c1w.cpu().numpy()) < 2e-5
    assert _rel(gotb, c1b.cpu().numpy()) < 2e-5


def test_conv12_bwd_route_in_the_train_step(cuda):
    """The step's k = 1 backward as one walk (CONV12_BWD=1, the default; the forward writes
    no y1) against the two-launch route (conv2's weight gradient on the forward's y1,
    CONV12_BWD=0), bench width, B = 32: every gradient but conv1's and conv2's kernel /
    bias bit-identical, those to the summation order (2e-5)."""
    import bench
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, options
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    img, width, lab = bench.synthetic_batch(np.random.default_rng(3), 32, 256, 125, cuda)
    out = []
    for route in (0, 1):
        store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=torch.bfloat16), device=cuda, seed=11)
        with options.override(CONV12_BWD=route):
            Trainer(store).loss_and_grads(img, width, lab)
        torch.cuda.synchronize()
        out.append({k: v.cpu().numpy().copy() for k, v in store.grads.items()})
    for k in out[0]:
        if k.startswith("convnet/conv1/") or k == "convnet/conv2/kernel":
            assert _rel(out[1][k], out[0][k]) < 2e-5, k
        else:
            np.testing.assert_array_equal(out[1][k], out[0][k], err_msg=k)


@pytest.mark.parametrize("M_,N,K,tag", [(8000, 4096, 256, "proj L1"), (8000, 4096, 1024, "proj L2"),
                                         (8000, 1024, 4096, "dx L2"), (8000, 256, 4096, "dx L1"),
                                         (8000, 1024, 96, "logits dx")])
def test_bf16_plain_gemms_bias_bf16_out(cuda, M_, N, K, tag):
    """The recurrent projection / data-gradient GEMMs with a bf16 C (the
    hand-written ping-pong engine for N >= 512, the NT engine below)."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(N + K)
    a = _bf(rng.standard_normal((M_, K)))
    w = _bf(rng.standard_normal((N, K)) / np.sqrt(K))
    bias = rng.standard_normal(N).astype(np.float32)
    ref = a.astype(np.float64) @ w.astype(np.float64).T + bias
    out = Kn.gemm(torch.from_numpy(a).to(cuda).bfloat16(), torch.from_numpy(w).to(cuda).bfloat16(), trans_b=True,
                  bias=torch.from_numpy(bias).to(cuda), out_dtype=torch.bfloat16)
    assert _rel(out.float().cpu().numpy(), ref) < BF16_OUT, tag
    # every element within its own bf16 rounding (+ accumulation noise)
    err = np.abs(out.float().cpu().numpy() - ref)
    assert np.all(err <= 2 ** -8 * np.abs(ref) + 1e-3 * np.abs(ref).max()), tag


@pytest.mark.parametrize("R,n_in,G4,splits,col", [(8000, 1024, 2048, 4, 0), (8000, 512, 2048, 8, 2048),
                                                   (8000, 256, 2048, 1, 0), (8000, 1024, 96, 3, 0),
                                                   (1000, 264, 296, 2, 8)])
def test_bf16_tn_weight_gradient_recurrent_shape(cuda, R, n_in, G4, splits, col):
    """dW = x^T . dG[:, col:col+G4] over T*B rows (the weight-gradient TN
    engines: ping-pong 256 x 256 for M, N >= 256, else 128-wide), split K and
    in-place f32 accumulation, ragged edges."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    rng = np.random.default_rng(3 + n_in)
    ld = max(2 * G4, col + G4)
    x = _bf(rng.standard_normal((R, n_in)))
    dG = _bf(rng.standard_normal((R, ld)))
    prev = rng.standard_normal((n_in, G4)).astype(np.float32)
    ref = prev + x.astype(np.float64).T @ dG[:, col:col + G4].astype(np.float64)
    gk = torch.from_numpy(prev).to(cuda)
    xd, dGd = torch.from_numpy(x).to(cuda).bfloat16(), torch.from_numpy(dG).to(cuda).bfloat16()
    Kn.gemm(xd, dGd[:, col:], trans_a=True, out=gk, accumulate=True, M=n_in, N=G4, K=R, lda=n_in, ldb=ld, ldc=G4,
            splits=splits)
    assert _rel(gk.cpu().numpy(), ref) < 1e-5


def _bf16_storage_oracle_grads(monkeypatch, vals, x, widths, labels, sizes):
    """The float64 oracle with every conv-tower op's output rounded to bf16
    (conv, BN, ReLU, max-pool and their backward ops): what bf16 STORAGE of
    the activations and gradients alone does to the exact result."""
    def wrap(f):
        def g(*a, **k):
            r = f(*a, **k)
            if isinstance(r, tuple):
                return tuple(_bf(v).astype(np.float64) if isinstance(v, np.ndarray) and v.ndim >= 3 else v
                             for v in r)
            return _bf(r).astype(np.float64) if isinstance(r, np.ndarray) else r
        return g
    for n in ("conv2d", "conv2d_bwd", "bn_train", "bn_bwd", "relu", "relu_bwd", "maxpool", "maxpool_bwd"):
        monkeypatch.setattr(G, n, wrap(getattr(G, n)))
    ref = M.RefModel({k: v.astype(np.float64) for k, v in vals.items()}, "lstm", sizes)
    out = ref.loss_and_grads(x, widths, labels)
    monkeypatch.undo()
    return out[1]


def test_bf16_train_step_bench_routes_vs_float64_oracle(cuda, monkeypatch):
    """One bf16 training forward + backward with every route of the bench
    (W=256, LSTM 512/512, persistent time loops, ping-pong projections),
    against the float64 oracle run on the bf16-rounded weights and inputs.
    Bounds: logits rel-L2 < 2e-2, mean CTC loss rel < 1e-3 (north_star), per-
    sequence loss rel < 1e-2, recurrent + logits gradients rel-L2 < 1e-2.
    The conv-tower gradients carry the error of bf16 activation storage
    itself, which grows down the tower through the BatchNorm backward
    (measured with the float64 oracle rounding its conv-tower op outputs to
    bf16: ~4e-2 at conv8 .. ~0.25 at conv1 at this random init); each conv
    variable's error must stay within 1.5x of that storage-only error (+1e-2)."""
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, model
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    B, W, sizes = 64, 256, (512, 512)
    rng = np.random.default_rng(2026)
    vals = M.init_params(seed=11, rnn_sizes=sizes)
    vals = {k: (_bf(v) if v.ndim >= 1 and "moving" not in k else v) for k, v in vals.items()}
    img = rng.integers(0, 256, (B, 32, W, 1)).astype(np.uint8)
    widths = np.full(B, W, np.int32)
    widths[1:8] = [250, 240, 230, 220, 210, 200, 190]
    labels = []
    for b in range(B):
        tl = G.seq_len_from_width([widths[b]])[0]
        while True:
            lab = list(rng.integers(0, 95, rng.integers(2, 20)))
            if G.ctc_required_time(lab) <= tl:
                break
        labels.append(lab)
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=sizes, dtype=torch.bfloat16), device=cuda, values=vals)
    store.zero_grad()
    feats, seq = model.convnet_layers(torch.from_numpy(img).to(cuda), torch.from_numpy(widths), model.TRAIN, store)
    logits = model.rnn_layers(feats, seq, 95, store)
    lab, ln = model.dense_labels(labels, B, cuda)
    loss_b, _, status = Kn.ctc_loss(logits.float().contiguous(), lab, ln, seq.to(torch.int32), need_grad=False)
    loss = model.ctc_loss_layer(logits, labels, seq)
    loss.backward()
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()

    x = G.preprocess(img).astype(np.float64)
    ref = M.RefModel({k: v.astype(np.float64) for k, v in vals.items()}, "lstm", sizes)
    loss_ref, grads_ref, losses_ref, logits_ref, seq_ref = ref.loss_and_grads(x, widths, labels)
    grads_emu = _bf16_storage_oracle_grads(monkeypatch, vals, x, widths, labels, sizes)
    assert seq.cpu().numpy().tolist() == seq_ref.tolist()
    lg = logits.detach().float().cpu().numpy()
    errs = {"logits": _rel(lg, logits_ref), "loss": abs(loss.item() - loss_ref) / abs(loss_ref),
            "loss_b": float(np.max(np.abs(loss_b.cpu().numpy() - losses_ref) / np.abs(losses_ref)))}
    bound = {}
    for name, g in grads_ref.items():
        got = store.grads[name].cpu().numpy()
        scale = np.linalg.norm(g)
        if name.endswith("/bias") and name.split("/")[1] in ("conv2", "conv4", "conv6", "conv8"):
            # a bias in front of BatchNorm: exactly zero gradient, both sides are rounding noise
            scale = max(scale, 1e-2 * np.linalg.norm(grads_ref[name.replace("/bias", "/kernel")]))
        errs[name] = float(np.linalg.norm(got - g) / max(scale, 1e-12))
        emu = float(np.linalg.norm(grads_emu[name] - g) / max(scale, 1e-12))
        bound[name] = 1e-2 if name.startswith("rnn/") else 1.5 * emu + 1e-2
    print("bf16 bench-route errors vs float64 oracle:", {k: f"{v:.2e}" for k, v in errs.items()})
    print("bounds (bf16-storage oracle):", {k: f"{v:.2e}" for k, v in bound.items()})
    assert errs["logits"] < 2e-2, errs
    assert errs["loss"] < 1e-3, errs
    assert errs["loss_b"] < 1e-2, errs
    bad = {k: (errs[k], bound[k]) for k in bound if errs[k] > bound[k]}
    assert not bad, bad


def _bench_batch(B, W, seed):
    """bench.py's synthetic C3 batch (uint8 crops, labels len U{2..19} fitting T)."""
    import bench
    T = (W - 2) // 2 - 2
    img, _w, (lab, ln) = bench.synthetic_batch(np.random.default_rng(seed), B, W, T, torch.device("cpu"))
    return img, lab, ln


@pytest.mark.parametrize("cell,sizes", [("lstm", (512, 512)), ("gru", (512, 256))])
def test_bf16_train_step_at_bench_shape_vs_float64(cuda, cell, sizes):
    """The benched step at the bench's OWN shape: B=256,
    W=256 (T*B = 32000 rows), the model's recurrent sizes, every default route
    -- the XCD-grouped persistent role map (B/8 % 16 == 0), the recurrent
    weight-gradient split-K counts of R = 32000 (model._splits), the batched
    direction-pair TN launches -- against the reference graph restated in
    PyTorch float64 on the host (oracle/torch_ref.py, pinned to the NumPy
    oracle to 1e-9 in tests/test_oracle.py) on the same bf16-rounded weights.
    cell="gru" is model.py's shipped GRU 512/256 (the bf16 GRU step
    and its gradients were unpinned).
    Bounds: mean CTC loss rel < 1e-3 (north_star), per-sequence loss rel < 1e-2,
    logits rel-L2 < 2e-2, recurrent + logits gradients rel-L2 < 1e-2; each conv
    variable within 1.5x (+1e-2) of the error that bf16 STORAGE of the conv
    tower's activations alone causes (the same float64 graph with those
    outputs and their gradients rounded to bf16)."""
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, model
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    from oracle.torch_ref import TorchRef
    B, W = 256, 256
    vals = M.init_params(seed=11, cell=cell, rnn_sizes=sizes)
    vals = {k: (_bf(v) if v.ndim >= 1 and "moving" not in k else v) for k, v in vals.items()}
    img, lab, ln = _bench_batch(B, W, 1234)
    store = ParamStore(ModelConfig(cell=cell, rnn_sizes=sizes, dtype=torch.bfloat16), device=cuda, values=vals)
    store.zero_grad()
    widths = torch.full((B,), W, dtype=torch.int32)
    feats, seq = model.convnet_layers(img.to(cuda), widths, model.TRAIN, store)
    logits = model.rnn_layers(feats, seq, 95, store)
    labd, lnd = lab.to(cuda), ln.to(cuda)
    loss_b, _, status = Kn.ctc_loss(logits.float().contiguous(), labd, lnd, seq.to(torch.int32), need_grad=False)
    loss = model.ctc_loss_layer(logits, (labd, lnd), seq)
    loss.backward()
    store.join()
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    v64 = {k: v.astype(np.float64) for k, v in vals.items()}
    lab64, ln64 = lab.long(), ln.long()
    loss_ref, grads_ref, losses_ref, logits_ref = TorchRef(v64, sizes, torch.float64, cell).loss_and_grads(
        img, lab64, ln64)
    _, grads_emu, _, _ = TorchRef(v64, sizes, torch.float64, cell, bf16_storage=True).loss_and_grads(img, lab64, ln64)
    lg = logits.detach().float().cpu().numpy()
    errs = {"logits": _rel(lg, logits_ref), "loss": abs(loss.item() - loss_ref) / abs(loss_ref),
            "loss_b": float(np.max(np.abs(loss_b.cpu().numpy() - losses_ref) / np.abs(losses_ref)))}
    bound = {}
    for name, g in grads_ref.items():
        got = store.grads[name].cpu().numpy()
        scale = np.linalg.norm(g)
        if name.endswith("/bias") and name.split("/")[1] in ("conv2", "conv4", "conv6", "conv8"):
            scale = max(scale, 1e-2 * np.linalg.norm(grads_ref[name.replace("/bias", "/kernel")]))
        errs[name] = float(np.linalg.norm(got - g) / max(scale, 1e-12))
        emu = float(np.linalg.norm(grads_emu[name] - g) / max(scale, 1e-12))
        bound[name] = 1e-2 if name.startswith("rnn/") else 1.5 * emu + 1e-2
    print(f"{cell} B=256 bf16 errors vs float64:", {k: f"{v:.2e}" for k, v in errs.items()})
    print("bounds (bf16-storage float64 graph):", {k: f"{v:.2e}" for k, v in bound.items()})
    assert errs["logits"] < 2e-2, errs
    assert errs["loss"] < 1e-3, errs
    assert errs["loss_b"] < 1e-2, errs
    bad = {k: (errs[k], bound[k]) for k in bound if errs[k] > bound[k]}
    assert not bad, bad


@pytest.mark.parametrize("cell,layer,items", [("lstm", 1, None), ("lstm", 2, None), ("gru", 1, None), ("gru", 2, None),
                                              ("lstm", 1, 128), ("lstm", 2, 128)])
def test_bf16_recurrent_weight_gradients_bench_launches(cuda, cell, layer, items):
    """The recurrent weight-gradient launches exactly as model._BiLSTM /
    _BiGRU.backward issue them at the bench's R = T*B = 32000 rows (batched
    direction pairs, stride_a / stride_b / stride_c, model._splits' split-K
    counts under the model's item caps, or a 128-item cap), into a non-zero
    f32 gradient (accumulate) -- against float64."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    from cnn_lstm_ctc_ocr_amd.model import _splits, _tn_items
    cap_x = items or _tn_items(layer)
    cap_h = items or _tn_items(layer)
    R = 32000
    H = 512 if (cell == "lstm" or layer == 1) else 256
    n_in = 256 if layer == 1 else (1024 if cell == "lstm" else 1024)
    G = 4 * H if cell == "lstm" else 2 * H            # LSTM gates / GRU r|u gates (the candidate block is H)
    ld = 2 * (4 * H if cell == "lstm" else 3 * H)
    rng = np.random.default_rng(layer * 10 + len(cell))
    x = _bf(rng.standard_normal((R, n_in)))
    hp = _bf(rng.standard_normal((R, 2 * H)))
    dG = _bf(rng.standard_normal((R, ld)) * 0.1)
    sk = (n_in + H) * G
    prev = rng.standard_normal(2 * sk).astype(np.float32)
    gk = torch.from_numpy(prev).to(cuda)
    xd, hd, dd = (torch.from_numpy(a).to(cuda).bfloat16() for a in (x, hp, dG))
    Kn.gemm(xd, dd, trans_a=True, out=gk, accumulate=True, M=n_in, N=G, K=R, lda=n_in, ldb=ld, ldc=G, batch=2,
            stride_a=0, stride_b=ld // 2, stride_c=sk, splits=_splits(n_in, G, R, batch=2, items=cap_x))
    Kn.gemm(hd, dd, trans_a=True, out=gk[n_in * G:], accumulate=True, M=H, N=G, K=R, lda=2 * H, ldb=ld, ldc=G,
            batch=2, stride_a=H, stride_b=ld // 2, stride_c=sk, splits=_splits(H, G, R, batch=2, items=cap_h))
    got = gk.cpu().numpy().reshape(2, n_in + H, G)
    x64, h64, d64 = x.astype(np.float64), hp.astype(np.float64), dG.astype(np.float64)
    for d in range(2):
        ref = prev[d * sk:(d + 1) * sk].reshape(n_in + H, G).astype(np.float64)
        dg = d64[:, d * (ld // 2):d * (ld // 2) + G]
        ref[:n_in] += x64.T @ dg
        ref[n_in:] += h64[:, d * H:(d + 1) * H].T @ dg
        assert _rel(got[d], ref) < 1e-5, (cell, layer, d, _splits(n_in, G, R, batch=2, items=cap_x),
                                          _splits(H, G, R, batch=2, items=cap_h))
