"""Run one batched weight-gradient (TN) GEMM as the train step issues it (for
rocprofv3 counter passes):  python tools/tn_one.py M N [reps]
(K = T*B = 32000, both directions as batch 2 over a [K][2N] dG, f32 C)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402
from cnn_lstm_ctc_ocr_amd.model import _splits  # noqa: E402

M, N = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
R = 32000
dev = torch.device("cuda")
x = (torch.rand(R, M, device=dev) * 2 - 1).bfloat16()
dG = (torch.rand(R, 2 * N, device=dev) * 2 - 1).bfloat16()
gk = torch.zeros(2, M, N, device=dev)
sp = _splits(M, N, R, batch=2)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for i in range(reps + 1):
    if i == 1:
        a.record()
    K.gemm(x, dG, trans_a=True, out=gk, accumulate=True, M=M, N=N, K=R, lda=M, ldb=2 * N, ldc=N, batch=2,
           stride_a=0, stride_b=N, stride_c=M * N, splits=sp)
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / reps
print(f"M={M} N={N} K={R} batch 2 splits {sp}: {ms * 1e3:.1f} us/call "
      f"{2 * 2.0 * M * N * R / ms / 1e9:.1f} TFLOP/s (incl. split-K reduce)", flush=True)
