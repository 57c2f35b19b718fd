"""Run one GEMM shape through K.gemm a few times (for rocprofv3 counter passes).

    python tools/pp_one.py M N K [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

M, N, Kd = (int(a) for a in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
dev = torch.device("cuda")
a = (torch.rand(M, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, Kd, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
bias = torch.randn(N, device=dev)
for _ in range(reps):
    K.gemm(a, w, trans_b=True, bias=bias, out_dtype=torch.bfloat16)
torch.cuda.synchronize()
print("done", flush=True)
