"""BN+ReLU+pool backward at the train step's four BN layers (diagnostic).
Run under rocprofv3 --kernel-trace --stats to split the passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402
from cnn_lstm_ctc_ocr_amd.config import POOLS  # noqa: E402

B = 256
LAYERS = [("conv2", 30, 254, 32), ("conv4", 15, 127, 64), ("conv6", 7, 126, 128), ("conv8", 3, 125, 256)]


def main():
    dev = torch.device("cuda")
    bf = torch.bfloat16
    for name, H, W, C in LAYERS:
        kh, kw, sh, sw = POOLS[name]
        Ho, Wo = (H - kh) // sh + 1, (W - kw) // sw + 1
        z = torch.randn(B, H, W, C, device=dev).to(bf)
        tm = name == "conv8"
        dp = torch.randn((Wo, B, C) if tm else (B, Ho, Wo, C), device=dev).to(bf)
        mean = torch.zeros(C, device=dev)
        inv = torch.ones(C, device=dev)
        g = torch.ones(C, device=dev)
        b = torch.zeros(C, device=dev)
        dg, db, dbias = (torch.zeros(C, device=dev) for _ in range(3))
        fn = lambda: K.bn_relu_pool_bwd(z, dp, mean, inv, g, b, (kh, kw, sh, sw), tm, dg, db, dbias=dbias)
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        mb = z.numel() * 2 / 1e6
        print(f"{name}: z {mb:7.1f} MB  {ms * 1e3:8.1f} us/call  ({3 * mb / ms / 1e3:6.2f} TB/s at 3x z)")


if __name__ == "__main__":
    main()
