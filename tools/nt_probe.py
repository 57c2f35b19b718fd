"""Where the NT engine's time goes on conv6-8 (the bench shape, B = 256):
the model's forward (implicit GEMM + BN statistics epilogue or ReLU), the same
without the statistics epilogue, and the same M x N x K as a plain row-major
GEMM on a materialised im2col matrix (no im2col address arithmetic, same
engine), each alone on the GPU.

    python tools/nt_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
B = 256
LAYERS = [("conv6", 7, 126, 128, 128, True), ("conv7", 3, 125, 128, 256, False), ("conv8", 3, 125, 256, 256, True)]


def timed(f, n=20):
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for name, H, W, cin, cout, bn in LAYERS:
    M = B * H * W
    fl = 2.0 * M * cout * 9 * cin
    x = (torch.rand(B, H, W, cin, device=dev) - 0.5).bfloat16()
    w_nk = (torch.rand(cout, 9 * cin, device=dev) - 0.5).bfloat16()
    bias = torch.rand(cout, device=dev)
    stats = torch.empty(K.conv_stats_tiles(M), 2, cout, device=dev)
    a = (torch.rand(M, 9 * cin, device=dev) - 0.5).bfloat16()
    res = {
        "model": timed(lambda: K.conv3x3_fwd(x, w_nk, bias, relu=not bn, stats=stats if bn else None)),
        "no-stats relu": timed(lambda: K.conv3x3_fwd(x, w_nk, bias, relu=True)),
        "with stats": timed(lambda: K.conv3x3_fwd(x, w_nk, bias, relu=False, stats=stats)),
        "plain GEMM (im2col materialised)": timed(lambda: K.gemm(a, w_nk, trans_b=True, bias=bias,
                                                                 out_dtype=torch.bfloat16)),
    }
    print(f"{name} M={M} N={cout} K={9 * cin}: " + "; ".join(f"{k} {v:.1f} us ({fl / v / 1e6:.0f} TF/s)"
                                                            for k, v in res.items()), flush=True)
