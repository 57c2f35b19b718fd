"""conv1 -> conv2's backward at the bench shape (B = 256, 30 x 254), each alone on the GPU:
the one-walk form (ocrk_conv12_bwd: backward-data + conv1's and conv2's weight gradients,
y1 recomputed) against the two launches it replaces (ocrk_conv2_bwd_data_conv1_wgrad, then
conv2's weight gradient on a stored y1).

    python tools/c12b_probe.py [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
B, IH, IW = 256, 32, 256
H, W = IH - 2, IW - 2
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randint(0, 256, (B, IH, IW), dtype=torch.uint8, device=dev, generator=g)
w1 = torch.randn(3, 3, 1, 32, device=dev, generator=g)
b1 = torch.randn(32, device=dev, generator=g) * 0.3
w2 = torch.randn(3, 3, 32, 32, device=dev, generator=g) / 17
w_nk = K.permute3(w2, 9 * 32, 32, 1, torch.bfloat16).view(32, 9 * 32)
w_bwd = K.permute3(w2, 9, 32, 32, torch.bfloat16).view(32, 9 * 32)
y1, bits, _, _ = K.conv12_fwd(x, w1, b1, w_nk, torch.zeros(32, device=dev))
dz = torch.randn(B, H, W, 32, device=dev, generator=g).bfloat16()
dw2, dw1, db1 = torch.zeros(3, 3, 32, 32, device=dev), torch.zeros(3, 3, 1, 32, device=dev), torch.zeros(32, device=dev)


def timed(f):
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


one = timed(lambda: K.conv12_bwd(dz, w_bwd, x, w1, b1, dw2, dw1, db1, relu_bits=bits))
dg = timed(lambda: K.conv2_bwd_data_conv1_wgrad(dz, w_bwd, None, x, dw1, db1, relu_bits=bits))
wg = timed(lambda: K.conv3x3_bwd_weight(y1, dz, dw2))
print(f"one walk (ocrk_conv12_bwd) {one:.1f} us; backward-data + conv1 dW {dg:.1f} us + conv2 dW {wg:.1f} us "
      f"= {dg + wg:.1f} us", flush=True)
