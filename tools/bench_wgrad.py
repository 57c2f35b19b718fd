"""Conv weight gradients of the train step (B=256, 32x256 crops) in isolation:
time per ocrk_conv3x3_bwd_weight call (whatever route the dispatcher picks:
row-walking, 4-wave TN, ping-pong TN im2col) and TFLOP/s."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
B = int(os.environ.get("B", "256"))
LAYERS = [("conv2", 30, 254, 32, 32), ("conv3", 15, 127, 32, 64), ("conv4", 15, 127, 64, 64),
          ("conv5", 7, 126, 64, 128), ("conv6", 7, 126, 128, 128), ("conv7", 3, 125, 128, 256),
          ("conv8", 3, 125, 256, 256)]
for name, H, W, cin, cout in LAYERS:
    x = (torch.rand(B, H, W, cin, device=dev) * 2 - 1).bfloat16()
    dy = (torch.rand(B, H, W, cout, device=dev) * 2 - 1).bfloat16()
    dw = torch.zeros(9 * cin, cout, device=dev)
    f = lambda: K.conv3x3_bwd_weight(x, dy, dw, accumulate=False)  # noqa: E731
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        f()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 10 * 1e3
    fl = 2.0 * B * H * W * 9 * cin * cout
    print(f"{name} {cin}->{cout}: {us:7.1f} us  {fl / us / 1e6:6.1f} TFLOP/s", flush=True)
