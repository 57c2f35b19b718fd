"""Per-layer conv timings of the bench shape (B=256, 32x256 crops): forward
(with the BN-statistics or ReLU epilogue the model uses) and backward-data
(with the ReLU mask / bias-gradient fusions the model uses), on the route the
dispatcher picks (OCRK_CONV_DIRECT=0: implicit GEMM only). Prints us,
TFLOP/s and the HBM-byte floor of each launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
B = int(os.environ.get("B", "256"))
# (layer, H, W, cin, cout, bn) at 32x256 input: conv1 valid -> 30x254, pools as model.py:111-145
LAYERS = [("conv2", 30, 254, 32, 32, True), ("conv3", 15, 127, 32, 64, False), ("conv4", 15, 127, 64, 64, True),
          ("conv5", 7, 126, 64, 128, False), ("conv6", 7, 126, 128, 128, True), ("conv7", 3, 125, 128, 256, False),
          ("conv8", 3, 125, 256, 256, True)]


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


tot_f = tot_d = tot_w = 0.0
for name, H, W, cin, cout, bn in LAYERS:
    M = B * H * W
    x = (torch.rand(B, H, W, cin, device=dev) - 0.5).bfloat16()
    w_nk = (torch.rand(cout, 9 * cin, device=dev) - 0.5).bfloat16()
    w_bwd = (torch.rand(cin, 9 * cout, device=dev) - 0.5).bfloat16()
    bias = torch.rand(cout, device=dev)
    stats = torch.empty(K.conv_stats_tiles(M), 2, cout, device=dev) if bn else None
    dy = (torch.rand(B, H, W, cout, device=dev) - 0.5).bfloat16()
    mask = (torch.rand(B, H, W, cin, device=dev) - 0.5).bfloat16() if bn else None
    dbias = torch.zeros(cin, device=dev) if (bn and name != "conv2") else None
    tf = timed(lambda: K.conv3x3_fwd(x, w_nk, bias, relu=not bn, stats=stats))
    if bn and K.conv3x3_fwd_rowstats_ok(x, cout):                   # the model's route for conv2
        tf = timed(lambda: K.conv3x3_fwd_rowstats(x, w_nk, bias))
    td = timed(lambda: K.conv3x3_bwd_data(dy, w_bwd, relu_mask=mask, dbias=dbias))
    dw = torch.zeros(3, 3, cin, cout, device=dev)
    tw = timed(lambda: K.conv3x3_bwd_weight(x, dy, dw))
    fl = 2.0 * M * cout * 9 * cin
    fb = M * (cin + cout) * 2
    tot_f += tf
    tot_d += td
    print(f"{name} M={M:8d} {cin:3d}->{cout:3d}  fwd {tf:7.1f} us {fl / tf / 1e6:7.1f} TF/s (HBM floor "
          f"{fb / 8e6:5.1f} us)   dgrad {td:7.1f} us {fl / td / 1e6:7.1f} TF/s   wgrad {tw:7.1f} us "
          f"{fl / tw / 1e6:7.1f} TF/s", flush=True)
    tot_w += tw
print(f"total fwd {tot_f:.1f} us  dgrad {tot_d:.1f} us  wgrad {tot_w:.1f} us")
