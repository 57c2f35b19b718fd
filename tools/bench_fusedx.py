"""The first layer's persistent forward, fused input projection vs projection
GEMM + loop (diagnostics): per-step time and the in-kernel stamps of step 64.
    python tools/bench_fusedx.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# debug stamps (include/ocrk_debug.h) live in the tools-only build: `make exp`
os.environ.setdefault("OCRK_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libocrk_exp.so"))
from cnn_lstm_ctc_ocr_amd import _lib, kernels as K  # noqa: E402

B, H, T, n_in = 256, 512, 125, 256
dev = torch.device("cuda")
torch.manual_seed(0)
x = (torch.randn(T, B, n_in, device=dev) * 0.5).bfloat16()
wxT = (torch.randn(8 * H, n_in, device=dev) * 0.05).bfloat16()
bias = torch.randn(8 * H, device=dev) * 0.1
whT = (torch.randn(2, 4 * H, H, device=dev) * 0.02).bfloat16()
seq = torch.full((B,), T, dtype=torch.int32, device=dev)


def unfused():
    gx = K.gemm(x.view(T * B, n_in), wxT, trans_b=True, bias=bias, out_dtype=torch.bfloat16)
    return K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)


def fused():
    return K.lstm_fwd_fused_x(x, wxT, bias, whT, seq, T, B, H)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


gx = K.gemm(x.view(T * B, n_in), wxT, trans_b=True, bias=bias, out_dtype=torch.bfloat16)
print(f"projection GEMM {timed(lambda: K.gemm(x.view(T * B, n_in), wxT, trans_b=True, bias=bias, out_dtype=torch.bfloat16)):.1f} us; "
      f"loop {timed(lambda: K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)):.1f} us; "
      f"GEMM + loop {timed(unfused):.1f} us; fused {timed(fused):.1f} us", flush=True)
names = ["top", "flags seen", "h staged", "gates spilled", "h published", "saved stored"]
for kind, fn in (("unfused loop", lambda: K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)), ("fused", fused)):
    dbg = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
    _lib.call("ocrk_lstm_debug_stamps", _lib.ptr(dbg))
    fn()
    torch.cuda.synchronize()
    _lib.call("ocrk_lstm_debug_stamps", None)
    grid = 2 * (B // 32) * (H // 32)
    st = dbg.view(-1, 8)[:grid].cpu().numpy().astype(np.float64) * 10.0
    seg = [st[:, i] for i in range(6)] + [st[:, 6]]
    print(f"{kind}: step 64 -> 65 median {np.median(st[:, 6] - st[:, 0]):.0f} ns")
    for i in range(6):
        d = seg[i + 1] - seg[i]
        nxt = names[i + 1] if i + 1 < 6 else "next step"
        print(f"  {names[i]:>14s} -> {nxt:<14s} median {np.median(d):7.0f} ns  p90 {np.percentile(d, 90):7.0f}")
