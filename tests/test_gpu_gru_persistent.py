"""The persistent bf16 BiGRU time loops (csrc/gru_persistent.hip, the default
for bf16 GRU layers) against the per-step kernels and the float64 oracle
(oracle/ref_graph.py gru_dir_fwd / gru_dir_bwd, restating
src/weinman/model.py:167-199 with [TF1] GRUCell): forward outputs and saved
tensors, and the BPTT gate gradients checked through the weight / bias
gradients they produce (dW_h = h_prev^T . dz, db = sum dz) -- at a small
shape and at the reference model.py's configuration GRU 512/256 with B = 256,
T = 125 (both layers' shapes), ragged sequence lengths."""
import numpy as np
import pytest
import torch

from oracle import ref_graph as G

pytestmark = pytest.mark.gpu


def _both(ocrk_opts, fn):
    ocrk_opts("LSTM_PERSISTENT", 0)
    step = fn()
    ocrk_opts("LSTM_PERSISTENT", 1)
    pers = fn()
    torch.cuda.synchronize()
    return step, pers


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("T,B,n_in,H", [(11, 64, 32, 256), (125, 256, 256, 512), (125, 256, 1024, 256)])
def test_gru_persistent_matches_step_kernels_and_oracle(cuda, ocrk_opts, T, B, n_in, H):
    from cnn_lstm_ctc_ocr_amd import kernels as K
    rng = np.random.default_rng(11 + H + n_in)
    bf = lambda a: torch.from_numpy(np.asarray(a, np.float32)).bfloat16().float().numpy()   # noqa: E731
    x = bf(rng.standard_normal((T, B, n_in)))
    sc = 1.0 / np.sqrt(n_in + H)
    gks = [bf(rng.standard_normal((n_in + H, 2 * H)) * 2 * sc) for _ in range(2)]
    cks = [bf(rng.standard_normal((n_in + H, H)) * 2 * sc) for _ in range(2)]
    gbs = [(1.0 + 0.1 * rng.standard_normal(2 * H)).astype(np.float32) for _ in range(2)]   # TF1 gate bias init 1
    cbs = [(0.1 * rng.standard_normal(H)).astype(np.float32) for _ in range(2)]
    seq = rng.integers(max(1, T // 2), T + 1, B).astype(np.int32)
    seq[:3] = [T, 1, T - 1]
    x64 = x.astype(np.float64)
    fw = [G.gru_dir_fwd(x64, seq, gks[d].astype(np.float64), gbs[d].astype(np.float64), cks[d].astype(np.float64),
                        cbs[d].astype(np.float64), d == 1) for d in range(2)]
    ref = np.concatenate([o for o, _ in fw], axis=2)

    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)   # noqa: E731
    wxT = np.concatenate([np.concatenate([gks[d][:n_in], cks[d][:n_in]], 1).T for d in range(2)], 0)   # [6H, n_in]
    bias = np.concatenate([np.concatenate([gbs[d], cbs[d]]) for d in range(2)])
    whgT = dev(np.stack([g[n_in:].T for g in gks])).bfloat16()
    whcT = dev(np.stack([c[n_in:].T for c in cks])).bfloat16()
    whg = dev(np.stack([g[n_in:] for g in gks])).bfloat16()
    whc = dev(np.stack([c[n_in:] for c in cks])).bfloat16()
    gx = K.gemm(dev(x.reshape(T * B, n_in)).bfloat16(), dev(wxT).bfloat16(), trans_b=True, bias=dev(bias),
                out_dtype=torch.bfloat16)
    seq_d = dev(seq)
    assert K.gru_persistent_ok(B, H, torch.bfloat16)
    K.status_word(cuda).zero_()
    step, pers = _both(ocrk_opts, lambda: K.gru_fwd(gx, whgT, whcT, seq_d, T, B, H, torch.bfloat16))
    assert K.read_status(cuda) == 0
    # both orders feed h back in bf16 and drift apart by a few bf16 ulps per step; the oracle bounds both
    for a, b in zip(step, pers):
        assert (a.float() - b.float()).abs().max().item() < 6e-2 * max(1.0, a.float().abs().max().item())
    out = pers[0].float().cpu().numpy()
    e_out = _rel(out, ref)
    assert e_out < 2e-2, e_out
    assert np.all(out[seq[1]:, 1] == 0)

    dout_np = bf(rng.standard_normal(ref.shape))
    dout = dev(dout_np).bfloat16()
    _, hprev, _rh, acts = pers
    dstep, dpers = _both(ocrk_opts, lambda: K.gru_bwd(whg, whc, seq_d, dout, hprev, acts, T, B, H))
    assert K.read_status(cuda) == 0
    scale = dstep.float().abs().max().item()
    assert (dstep.float() - dpers.float()).abs().max().item() < 3e-2 * max(scale, 1e-6)
    # the gate gradients through what the train step makes of them, against float64 BPTT
    dG = dpers.float().cpu().numpy().astype(np.float64)                  # [T, B, 2, 3H]
    hp = hprev.float().cpu().numpy().astype(np.float64)                  # [T, B, 2, H]
    errs = {}
    for d in range(2):
        _dx, dgk, dgb, dck, dcb = G.gru_dir_bwd(dout_np[:, :, d * H:(d + 1) * H].astype(np.float64), fw[d][1],
                                                gks[d].astype(np.float64), cks[d].astype(np.float64), n_in)
        dzg = dG[:, :, d, :2 * H].reshape(T * B, 2 * H)
        dzc = dG[:, :, d, 2 * H:].reshape(T * B, H)
        errs[f"d{d}/gates/bias"] = _rel(dzg.sum(0), dgb)
        errs[f"d{d}/candidate/bias"] = _rel(dzc.sum(0), dcb)
        errs[f"d{d}/gates/W_h"] = _rel(hp[:, :, d].reshape(T * B, H).T @ dzg, dgk[n_in:])
        errs[f"d{d}/gates/W_x"] = _rel(x64.reshape(T * B, n_in).T @ dzg, dgk[:n_in])
        errs[f"d{d}/candidate/W_x"] = _rel(x64.reshape(T * B, n_in).T @ dzc, dck[:n_in])
    print("persistent GRU vs float64 BPTT:", errs, "out", e_out)
    assert max(errs.values()) < 2e-2, errs


def test_gru_persistent_timeout_sets_status_and_raises(cuda, ocrk_opts):
    """A hand-off wait that gives up (spin limit forced to 1 poll) ORs its bit
    into the status word, the launch still completes, the host raises."""
    from cnn_lstm_ctc_ocr_amd import _lib
    from cnn_lstm_ctc_ocr_amd import kernels as K
    T, B, H = 32, 256, 512
    torch.manual_seed(0)
    gx = (torch.randn(T * B, 6 * H, device=cuda) * 0.1).bfloat16()
    whgT = (torch.randn(2, 2 * H, H, device=cuda) * 0.02).bfloat16()
    whcT = (torch.randn(2, H, H, device=cuda) * 0.02).bfloat16()
    seq = torch.full((B,), T, dtype=torch.int32, device=cuda)
    assert K.gru_persistent_ok(B, H, torch.bfloat16)
    K.status_word(cuda).zero_()
    ocrk_opts("LSTM_SPIN_LIMIT", 1)
    K.gru_fwd(gx, whgT, whcT, seq, T, B, H, torch.bfloat16)
    torch.cuda.synchronize()
    ocrk_opts.reset("LSTM_SPIN_LIMIT")
    with pytest.raises(_lib.DeviceError):
        K.check_status(cuda)
    K.gru_fwd(gx, whgT, whcT, seq, T, B, H, torch.bfloat16)
    assert K.read_status(cuda) == 0
