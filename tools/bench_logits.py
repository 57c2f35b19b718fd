"""The logits forward GEMM (model.py:216-220: [T*B, 1024] . W^T + b, ReLU, f32
out, N = 96) and the layer-1 data gradient (N = 256, K = 4096) at the bench
shape, per launch (diagnostic; OCRK_GEMM_NT_CFG picks a tile config)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


dev = torch.device("cuda")
torch.manual_seed(0)
x = (torch.rand(32000, 1024, device=dev) - 0.5).bfloat16()
wT = (torch.rand(96, 1024, device=dev) - 0.5).bfloat16()
bias = torch.rand(96, device=dev)
t1 = timed(lambda: K.gemm(x, wT, trans_b=True, bias=bias, relu=True))
dg = (torch.rand(32000, 4096, device=dev) - 0.5).bfloat16()
wx = (torch.rand(256, 4096, device=dev) - 0.5).bfloat16()
t2 = timed(lambda: K.gemm(dg, wx, trans_b=True, out_dtype=torch.bfloat16))
cfg = os.environ.get("OCRK_GEMM_NT_CFG", "-1")
print(f"cfg {cfg:>3s}: logits fwd {t1:6.1f} us ({2 * 32000 * 96 * 1024 / t1 / 1e6:5.0f} TF/s)   "
      f"dx L1 {t2:6.1f} us ({2 * 32000 * 256 * 4096 / t2 / 1e6:5.0f} TF/s)", flush=True)
