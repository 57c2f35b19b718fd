"""conv1 -> conv2 forward at the bench shape (B = 256, 32 x 256 u8 crops), alone on the GPU:
ocrk_conv12_fwd without y1 (the training route) and with it.

    python tools/c12f_probe.py [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
B, IH, IW = 256, 32, 256
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randint(0, 256, (B, IH, IW), dtype=torch.uint8, device=dev, generator=g)
w1 = torch.randn(3, 3, 1, 32, device=dev, generator=g)
b1 = torch.randn(32, device=dev, generator=g) * 0.3
w2 = torch.randn(3, 3, 32, 32, device=dev, generator=g) / 17
w_nk = K.permute3(w2, 9 * 32, 32, 1, torch.bfloat16).view(32, 9 * 32)
b2 = torch.zeros(32, device=dev)


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


t0 = timed(lambda: K.conv12_fwd(x, w1, b1, w_nk, b2, want_y1=False))
t1 = timed(lambda: K.conv12_fwd(x, w1, b1, w_nk, b2, want_y1=True))
print(f"conv12 forward: no y1 {t0:.1f} us, with y1 {t1:.1f} us", flush=True)
