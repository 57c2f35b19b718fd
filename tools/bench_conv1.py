"""conv1 (fused preprocess) forward and weight gradient of the bench step in
isolation (B=256 crops of 32x256 uint8 -> [256, 30, 254, 32] bf16), with the
HBM-byte floor of each: forward writes the output, the weight gradient reads dz."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
B, H, W, C = int(os.environ.get("B", "256")), 32, int(os.environ.get("W", "256")), 32


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


x = torch.randint(0, 256, (B, H, W), dtype=torch.uint8, device=dev)
w, bias = torch.randn(3, 3, 1, C, device=dev) * 0.3, torch.randn(C, device=dev) * 0.1
y = K.conv1_fwd(x, w, bias, torch.bfloat16)
dz = torch.randn_like(y)
dw, db = torch.zeros(3, 3, 1, C, device=dev), torch.zeros(C, device=dev)
tf = timed(lambda: K.conv1_fwd(x, w, bias, torch.bfloat16))
tw = timed(lambda: K.conv1_bwd_weight(x, dz, dw, db, accumulate=False))
yb = y.numel() * 2
print(f"conv1 y {tuple(y.shape)}  fwd {tf:7.1f} us (floor {yb / 8e6:5.1f})   wgrad {tw:7.1f} us (floor {yb / 8e6:5.1f})",
      flush=True)
