"""Probe the ping-pong engine's ReLU-mask epilogue (experiments build, OCRK_GEMM_PP=2)
with structured masks: constant, channel-alternating, pixel-alternating."""
import sys

sys.path.insert(0, "/root/repo")
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(3)
B, H, W, cin, cout = 16, 7, 126, 128, 128
dy = torch.randn(B, H, W, cout, device=dev, generator=g).bfloat16()
w = (torch.randn(3, 3, cin, cout, device=dev, generator=g) / 30).bfloat16()
w_bwd = w.permute(2, 0, 1, 3).contiguous().view(cin, 9 * cout)
ref = K.conv3x3_bwd_data(dy, w_bwd)
ch = torch.arange(cin, device=dev)
px = torch.arange(B * H * W, device=dev).view(B, H, W, 1)
masks = [("chan_even", (ch % 2 == 0).float().expand(B, H, W, cin) * 2 - 1),
         ("chan_lt64", (ch < 64).float().expand(B, H, W, cin) * 2 - 1),
         ("chan_mod4_0", (ch % 4 == 0).float().expand(B, H, W, cin) * 2 - 1),
         ("pix_even", (px % 2 == 0).float().expand(B, H, W, cin) * 2 - 1)]
for name, m in masks:
    m = m.contiguous().bfloat16()
    dx = K.conv3x3_bwd_data(dy, w_bwd, relu_mask=m)
    keep = (dx.float() != 0).view(-1, cin)
    exp = (m.float() > 0).view(-1, cin)
    print(name, "mismatched keep pattern:", int((keep != exp).sum()), "of", keep.numel(), flush=True)
    print("  pixel 0 kept channels (got):", keep[0, :16].int().tolist())
    print("  pixel 0 kept channels (exp):", exp[0, :16].int().tolist())
    print("  pixel 1 kept channels (got):", keep[1, :16].int().tolist(), flush=True)
