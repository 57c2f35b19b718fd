"""BN + ReLU + max-pool forward / backward of the bench step's four BN layers
in isolation (B=256, 32x256 crops), with the HBM-byte floor of each call:
forward reads z and writes the pooled output; backward reads z and dp,
writes dz (plus the routed-gradient image it stages internally)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
B = int(os.environ.get("B", "256"))
# (layer, H, W, C, pool (kh, kw, sh, sw), time-major output)
LAYERS = [("conv2", 30, 254, 32, (2, 2, 2, 2), False), ("conv4", 15, 127, 64, (2, 2, 2, 1), False),
          ("conv6", 7, 126, 128, (2, 2, 2, 1), False), ("conv8", 3, 125, 256, (3, 1, 3, 1), True)]


def timed(f, n=10):
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for name, H, W, C, pool, tm in LAYERS:
    z = torch.randn(B, H, W, C, device=dev).bfloat16()
    mean, invstd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    y = K.bn_relu_pool_fwd(z, mean, invstd, gamma, beta, pool, time_major=tm)
    dp = torch.randn_like(y)
    dg, db, dbias = torch.zeros(C, device=dev), torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    tf = timed(lambda: K.bn_relu_pool_fwd(z, mean, invstd, gamma, beta, pool, time_major=tm))
    tb = timed(lambda: K.bn_relu_pool_bwd(z, dp, mean, invstd, gamma, beta, pool, tm, dg, db, dbias=dbias))
    tp = timed(lambda: K.bn_relu_pool_bwd(z, dp, mean, invstd, gamma, beta, pool, tm, dg, db, dbias=dbias, pooled=y))
    zb, yb = z.numel() * 2, y.numel() * 2
    print(f"{name} z {tuple(z.shape)}  fwd {tf:7.1f} us (floor {(zb + yb) / 8e6:5.1f})   "
          f"bwd {tb:7.1f} us (floor {(2 * zb + yb) / 8e6:5.1f}; staged da image +{2 * zb / 8e6:.1f})   "
          f"bwd pooled {tp:7.1f} us", flush=True)
