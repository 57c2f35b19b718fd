"""The persistent bf16 BiLSTM forward (opt-in) against the per-step kernels and the oracle."""
import numpy as np
import pytest
import torch

from oracle import ref_graph as G

pytestmark = pytest.mark.gpu


def test_persistent_matches_step_kernels_and_oracle(cuda, monkeypatch):
    from cnn_lstm_ctc_ocr_amd import kernels as K
    rng = np.random.default_rng(7)
    T, B, n_in, H = 11, 64, 32, 256
    x = torch.from_numpy(rng.standard_normal((T, B, n_in)).astype(np.float32)).bfloat16().float().numpy()
    ks = [torch.from_numpy((rng.standard_normal((n_in + H, 4 * H)) * 0.2).astype(np.float32)).bfloat16().float().numpy()
          for _ in range(2)]
    bs = [(rng.standard_normal(4 * H) * 0.2).astype(np.float32) for _ in range(2)]
    seq = rng.integers(1, T + 1, B).astype(np.int32)
    seq[:3] = [T, 1, T - 1]
    ref = np.concatenate([G.lstm_dir_fwd(x, seq, ks[d], bs[d], d == 1)[0] for d in range(2)], axis=2)
    wxT = np.ascontiguousarray(np.concatenate([k[:n_in].T for k in ks], 0))
    whT = np.ascontiguousarray(np.stack([k[n_in:].T for k in ks]))
    gx = K.gemm(torch.from_numpy(x.reshape(T * B, n_in)).to(cuda).bfloat16(),
                torch.from_numpy(wxT).to(cuda).bfloat16(), trans_b=True,
                bias=torch.from_numpy(np.concatenate(bs)).to(cuda), out_dtype=torch.bfloat16)
    whT_d = torch.from_numpy(whT).to(cuda).bfloat16()
    seq_d = torch.from_numpy(seq).to(cuda)
    monkeypatch.setenv("OCRK_LSTM_PERSISTENT", "0")
    K._PERSISTENT.clear()
    step = K.lstm_fwd(gx, whT_d, seq_d, T, B, H, torch.bfloat16)
    monkeypatch.setenv("OCRK_LSTM_PERSISTENT", "1")
    K._PERSISTENT.clear()
    assert K.lstm_persistent_ok(B, H, torch.bfloat16)
    K.lstm_error_word(cuda).zero_()
    pers = K.lstm_fwd(gx, whT_d, seq_d, T, B, H, torch.bfloat16)
    torch.cuda.synchronize()
    K._PERSISTENT.clear()
    assert K.lstm_error_word(cuda).item() == 0
    for a, b in zip(step, pers):
        assert (a.float() - b.float()).abs().max().item() < 2e-2
    out = pers[0].float().cpu().numpy()
    assert np.linalg.norm(out - ref) / np.linalg.norm(ref) < 3e-2
    assert np.all(out[seq[1]:, 1] == 0)
