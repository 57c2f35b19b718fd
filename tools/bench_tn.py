"""Weight-gradient (TN) GEMMs of the train step: time per call and TFLOP/s on
the engine the dispatcher picks (OCRK_GEMM_PPTN=0: the 4-wave engine)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402
from cnn_lstm_ctc_ocr_amd.model import _splits  # noqa: E402

R = 32000
dev = torch.device("cuda")
tot = 0.0
for n_in, N, ldb, tag in [(1024, 2048, 4096, "L2 dW_x (per dir)"), (512, 2048, 4096, "dW_h (per dir)"),
                          (256, 2048, 4096, "L1 dW_x (per dir)"), (1024, 96, 96, "logits dW")]:
    x = (torch.rand(R, n_in, device=dev) * 2 - 1).bfloat16()
    dG = (torch.rand(R, ldb, device=dev) * 2 - 1).bfloat16()
    gk = torch.zeros(n_in, N, device=dev)
    sp = _splits(n_in, N, R)
    f = lambda: K.gemm(x, dG, trans_a=True, out=gk, accumulate=True, M=n_in, N=N, K=R, lda=n_in, ldb=ldb,  # noqa: E731
                       ldc=N, splits=sp)
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        f()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    tot += ms * (4 if "dir" in tag else 1)
    print(f"{tag:20s} splits {sp:3d} {ms * 1e3:8.1f} us {2.0 * n_in * N * R / ms / 1e9:8.1f} TFLOP/s", flush=True)
print(f"per-step total (x4 for the per-direction GEMMs of both layers' dW_x / dW_h): {tot:.3f} ms")
