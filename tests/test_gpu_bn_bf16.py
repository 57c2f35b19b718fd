"""bf16 BN -> ReLU -> max-pool backward (csrc/bn.hip: bn_bwd_route_kernel,
bn_bwd_apply_kernel) against the float64 oracle (oracle/ref_graph.py bn_bwd,
maxpool_bwd, relu_bwd restating src/weinman/model.py:105-123 with [TF1]
MaxPoolGrad's first-max routing), on the bench step's four BN layers (pool
2x2/[2,2], 2x2/[2,1] x2, [3,1]/[3,1] time-major) at a reduced batch, plus
odd widths / uncovered rows / columns."""
import numpy as np
import pytest
import torch

from oracle import ref_graph as G

pytestmark = pytest.mark.gpu

CASES = [  # (B, H, W, C, pool)
    (4, 30, 254, 32, (2, 2, 2, 2)),
    (4, 15, 127, 64, (2, 2, 2, 1)),
    (4, 7, 126, 128, (2, 2, 2, 1)),
    (4, 3, 125, 256, (3, 1, 3, 1)),
    (3, 7, 37, 32, (2, 2, 2, 2)),       # odd width: an uncovered column; H = 7: an uncovered row
    (3, 9, 11, 64, (2, 2, 2, 1)),
    (2, 3, 9, 512, (3, 1, 3, 1)),
]


def _bf(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).bfloat16().float().numpy()


@pytest.mark.parametrize("pooled", [False, True])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:4])) + f"-p{''.join(map(str, c[4]))}")
def test_bn_bwd_bf16_vs_oracle(cuda, case, pooled):
    """pooled: the dgamma / dbeta pass streams the forward's pooled output and dp
    (ocrk_bn_relu_pool_bwd_pooled; xhat at each window's max recovered from the bf16
    output for the dz correction term, dgamma itself summed from z in the apply walk)."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    B, H, W, C, pool = case
    rng = np.random.default_rng(B * H + W + C)
    z = _bf(rng.standard_normal((B, H, W, C)) * 1.5 + 0.3)
    gamma = (rng.random(C) + 0.5).astype(np.float32)
    beta = (rng.standard_normal(C) * 0.2).astype(np.float32)
    a, mean, var, _var_u, cache = G.bn_train(z.astype(np.float64), gamma.astype(np.float64), beta.astype(np.float64))
    tm = pool == (3, 1, 3, 1)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(cuda)   # noqa: E731
    mean_d = t(mean)
    inv_d = t(1 / np.sqrt(var + 1e-3))
    zd = t(z).bfloat16()
    p = Kn.bn_relu_pool_fwd(zd, mean_d, inv_d, t(gamma), t(beta), pool, time_major=tm)
    dp = _bf(rng.standard_normal(p.shape))
    dpd = t(dp).bfloat16()

    dg, db = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
    dbias = torch.zeros(C, device=cuda)
    dz = Kn.bn_relu_pool_bwd(zd, dpd, mean_d, inv_d, t(gamma), t(beta), pool, tm, dg, db, accumulate=False, dbias=dbias,
                             pooled=p if pooled else None)
    torch.cuda.synchronize()
    got = dz.float().cpu().numpy(), dg.cpu().numpy(), db.cpu().numpy(), dbias.cpu().numpy()
    scale = np.abs(got[0]).max()

    # float64 oracle on the same bf16 inputs (the routing is recomputed from the device's bf16 z)
    y = G.relu(a)
    dp_nchw = dp.transpose(1, 0, 2)[:, None] if tm else dp
    dy = G.maxpool_bwd(y, dp_nchw.astype(np.float64), *pool)
    dz_ref, dg_ref, db_ref = G.bn_bwd(G.relu_bwd(y, dy), cache, gamma.astype(np.float64))
    rel = lambda x, r: float(np.linalg.norm(x - r) / max(np.linalg.norm(r), 1e-30))   # noqa: E731
    assert rel(got[0], dz_ref) < 1e-2
    assert rel(got[1], dg_ref) < 1e-3
    assert rel(got[2], db_ref) < 1e-3
    assert np.abs(got[3] - dz_ref.sum(axis=(0, 1, 2))).max() <= 1e-3 * scale * np.sqrt(B * H * W)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", CASES[:4], ids=lambda c: "x".join(map(str, c[:4])))
def test_bn_bwd_pooled_matches_z_form(cuda, case, dtype):
    """The pooled-output pass 1 against the z walk on the same inputs: dbeta is the
    same terms (another order), dgamma is summed from z in both; dz differs only
    through sum(da * xhat), whose xhat the pooled form recovers as (p - beta) / gamma
    (bf16 p: ~2^-9 per term, so the correction term moves by ~1e-3 of itself; f32 p:
    rounding level). Also the deferred form: [bias | dgamma] partial rows summed by
    the caller give the same dbias / dgamma."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    B, H, W, C, pool = case
    rng = np.random.default_rng(7 * C + W)
    tm = pool == (3, 1, 3, 1)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(cuda)   # noqa: E731
    z = t(rng.standard_normal((B, H, W, C)) * 1.5 + 0.3).to(dtype)
    mean, inv = t(rng.standard_normal(C) * 0.1 + 0.3), t(rng.random(C) * 0.3 + 0.5)
    gamma, beta = t(rng.random(C) + 0.5), t(rng.standard_normal(C) * 0.2)
    p = Kn.bn_relu_pool_fwd(z, mean, inv, gamma, beta, pool, time_major=tm)
    dp = t(rng.standard_normal(p.shape)).to(dtype)
    outs = []
    for form in ("z", "pooled", "pooled-deferred"):
        dg, db, dbias = (torch.zeros(C, device=cuda) for _ in range(3))
        late = [] if form == "pooled-deferred" else None
        dz = Kn.bn_relu_pool_bwd(z, dp, mean, inv, gamma, beta, pool, tm, dg, db, accumulate=False, dbias=dbias,
                                 defer=late, pooled=None if form == "z" else p)
        for fn, _ in late or []:
            fn()
        torch.cuda.synchronize()
        outs.append((dz.double().cpu().numpy(), dg.double().cpu().numpy(), db.double().cpu().numpy(),
                     dbias.double().cpu().numpy()))
    rel = lambda x, r: float(np.linalg.norm(x - r) / max(np.linalg.norm(r), 1e-30))   # noqa: E731
    ref = outs[0]
    dz_tol = 4e-3 if dtype == torch.bfloat16 else 1e-5
    for got in outs[1:]:
        assert rel(got[0], ref[0]) < dz_tol
        assert rel(got[1], ref[1]) < 1e-5                 # dgamma: from z in both forms
        assert rel(got[2], ref[2]) < 1e-5                 # dbeta: the same terms
        # dbias = sum dz = -gamma invstd bm sum(xhat) here (mean is not z's batch mean, so
        # sum(xhat) != 0): it moves with bm itself; bounded like the oracle test's dbias
        scale = np.abs(ref[0]).max()
        assert np.abs(got[3] - ref[3]).max() <= (1e-3 if dtype == torch.bfloat16 else 1e-5) * scale * np.sqrt(B * H * W)
    np.testing.assert_array_equal(outs[1][0], outs[2][0])   # deferral moves no dz bit
    np.testing.assert_allclose(outs[2][1], outs[1][1], rtol=1e-6, atol=1e-6 * np.abs(outs[1][1]).max())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", CASES[:4], ids=lambda c: "x".join(map(str, c[:4])))
def test_bn_bwd_pooled_ill_conditioned_channels(cuda, case, dtype):
    """Channels where xhat = (p - beta) / gamma is ill-conditioned (|gamma| 1e-3..1e-2
    beside |beta| 0.5..2, gamma = 0, negative gamma) take the z walk's per-window terms
    inside the pooled pass (the stored output's rounding is amplified by
    |beta| / |gamma|, ~10 % at gamma = 0.01, beta = 0.5 in bf16). Those channels' dz
    must match the z form to summation order; the well-conditioned ones as before."""
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    B, H, W, C, pool = case
    rng = np.random.default_rng(11 * C + W)
    tm = pool == (3, 1, 3, 1)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(cuda)   # noqa: E731
    z = t(rng.standard_normal((B, H, W, C)) * 1.5 + 0.3).to(dtype)
    mean, inv = t(rng.standard_normal(C) * 0.1 + 0.3), t(rng.random(C) * 0.3 + 0.5)
    gamma = rng.random(C) + 0.5
    beta = rng.standard_normal(C) * 0.2
    ill = np.zeros(C, bool)
    ill[1::4] = True                                  # every 8-channel group holds some
    gamma[ill] = rng.uniform(1e-3, 1e-2, ill.sum()) * rng.choice([-1, 1], ill.sum())
    beta[ill] = rng.uniform(0.5, 2.0, ill.sum())
    gamma[5] = 0.0
    ill[5] = True
    gamma[2] = -gamma[2]                              # negative, well-conditioned
    gamma, beta = t(gamma), t(beta)
    p = Kn.bn_relu_pool_fwd(z, mean, inv, gamma, beta, pool, time_major=tm)
    dp = t(rng.standard_normal(p.shape)).to(dtype)
    outs = []
    for pooled in (None, p):
        dg, db, dbias = (torch.zeros(C, device=cuda) for _ in range(3))
        dz = Kn.bn_relu_pool_bwd(z, dp, mean, inv, gamma, beta, pool, tm, dg, db, accumulate=False, dbias=dbias,
                                 pooled=pooled)
        torch.cuda.synchronize()
        outs.append((dz.double().cpu().numpy().reshape(-1, C), dg.double().cpu().numpy(), db.double().cpu().numpy()))
    (zr, gr, br), (zp, gp, bp) = outs
    per = np.linalg.norm(zp - zr, axis=0) / np.maximum(np.linalg.norm(zr, axis=0), 1e-30)
    # the z form's own terms (another summation order; for the overlapping 2x2/[2,1] pool the
    # z form stages da in bf16 for its streaming apply, 2^-9 per routed sum -- hence bf16's 4e-3);
    # the (p - beta) / gamma recovery would be off by ~|beta| / |gamma| * 2^-9 = 10-200 % here
    tol = 4e-3 if dtype == torch.bfloat16 else 1e-5
    assert per[ill].max() < tol, per[ill]
    assert per[~ill].max() < tol, per[~ill]
    np.testing.assert_allclose(gp, gr, rtol=1e-5, atol=1e-5 * np.abs(gr).max())
    np.testing.assert_allclose(bp, br, rtol=1e-5, atol=1e-5 * np.abs(br).max())


def test_bn_bwd_pooled_defer_without_route(cuda):
    """with the window walk off (BN_ROUTE=0) the library takes the z form
    for a pooled call; the deferred bias slab must then have the z form's rows, and
    dbias / dgamma equal the undeferred z form's (ocrk_bn_bwd_pooled_bias_slab_rows
    == 0 tells the wrapper so; a pooled bias slab is refused by the C entry)."""
    from cnn_lstm_ctc_ocr_amd import _lib, options
    from cnn_lstm_ctc_ocr_amd import kernels as Kn
    B, H, W, C, pool = CASES[1]
    rng = np.random.default_rng(3)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(cuda)   # noqa: E731
    z = t(rng.standard_normal((B, H, W, C))).bfloat16()
    mean, inv = t(rng.standard_normal(C) * 0.1), t(rng.random(C) * 0.3 + 0.5)
    gamma, beta = t(rng.random(C) + 0.5), t(rng.standard_normal(C) * 0.2)
    p = Kn.bn_relu_pool_fwd(z, mean, inv, gamma, beta, pool)
    dp = t(rng.standard_normal(p.shape)).bfloat16()
    with options.override(BN_ROUTE=0):
        assert _lib.lib().ocrk_bn_bwd_pooled_bias_slab_rows(B, H, W, C, *pool) == 0
        res = []
        for pooled, late in ((None, None), (p, [])):
            dg, db, dbias = (torch.zeros(C, device=cuda) for _ in range(3))
            dz = Kn.bn_relu_pool_bwd(z, dp, mean, inv, gamma, beta, pool, False, dg, db, accumulate=False,
                                     dbias=dbias, defer=late, pooled=pooled)
            for fn, _ in late or []:
                fn()
            torch.cuda.synchronize()
            res.append([v.double().cpu().numpy() for v in (dz, dg, db, dbias)])
        slab = torch.empty(64, 2 * C, device=cuda)
        with pytest.raises(RuntimeError, match="pooled form is off"):
            Kn.call("ocrk_bn_relu_pool_bwd_pooled", Kn.ptr(z), Kn.ptr(p), Kn.ptr(dp), B, H, W, C, Kn.ptr(mean),
                    Kn.ptr(inv), Kn.ptr(gamma), Kn.ptr(beta), *pool, 0, Kn.ptr(torch.empty_like(z)),
                    Kn.ptr(torch.zeros(C, device=cuda)), Kn.ptr(torch.zeros(C, device=cuda)), None, 0,
                    Kn.ptr(slab), Kn.ptr(torch.empty(1 << 24, dtype=torch.uint8, device=cuda)), 1 << 24,
                    Kn.dtype_code(z.dtype), Kn._stream(z))
    for a, b in zip(*res):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6 * max(np.abs(b).max(), 1e-30))
