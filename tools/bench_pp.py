"""Ping-pong GEMM engine (csrc/gemm_pp.hip) on the train step's shapes:
time per launch, TFLOP/s and the error against a float32 torch reference
computed from the same bf16 operands (diagnostic; the parity tests are in
tests/).

    python tools/bench_pp.py                 # default routing (engine on)
    OCRK_GEMM_PP=0 python tools/bench_pp.py  # previous engines (hipBLASLt / NT)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

B = 256
CONV = [(30, 254, 32, 32), (15, 127, 32, 64), (15, 127, 64, 64), (7, 126, 64, 128), (7, 126, 128, 128),
        (3, 125, 128, 256), (3, 125, 256, 256)]


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def rel(x, ref):
    return float((x.float() - ref).norm() / ref.norm().clamp_min(1e-30))


def main():
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    torch.manual_seed(0)
    dev = torch.device("cuda")
    bf = torch.bfloat16
    rows = []
    for (M, N, Kd, tag) in [(32000, 4096, 256, "proj L1"), (32000, 4096, 1024, "proj L2"),
                            (32000, 1024, 4096, "dx L2"), (32000, 256, 4096, "dx L1"),
                            (32000, 1024, 96, "logits dx")]:
        if only and only not in tag:
            continue
        a = (torch.rand(M, Kd, device=dev) * 2 - 1).to(bf)
        w = ((torch.rand(N, Kd, device=dev) * 2 - 1) * 0.05).to(bf)
        bias = torch.randn(N, device=dev)
        out = K.gemm(a, w, trans_b=True, bias=bias, out_dtype=bf)
        ref = a.float() @ w.float().t() + bias
        ms = timed(lambda: K.gemm(a, w, trans_b=True, bias=bias, out_dtype=bf))
        rows.append((tag, ms, 2.0 * M * N * Kd, rel(out, ref)))
    for (H, W, Ci, Co) in ([] if only else CONV):
        x = (torch.rand(B, H, W, Ci, device=dev) * 2 - 1).to(bf)
        w = ((torch.rand(Co, 3, 3, Ci, device=dev) * 2 - 1) * 0.05).to(bf)          # [Cout][kh][kw][Cin]
        w_nk = w.reshape(Co, 9 * Ci).contiguous()
        bias = torch.randn(Co, device=dev)
        fl = 2.0 * B * H * W * 9 * Ci * Co
        y = K.conv3x3_fwd(x, w_nk, bias, relu=True)
        ref = F.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias, padding=1))
        err = rel(y.permute(0, 3, 1, 2), ref)
        ms = timed(lambda: K.conv3x3_fwd(x, w_nk, bias, relu=True))
        rows.append((f"conv fwd {Ci}->{Co} {H}x{W}", ms, fl, err))
        dy = (torch.rand(B, H, W, Co, device=dev) * 2 - 1).to(bf)
        w_bwd = w.permute(3, 1, 2, 0).reshape(Ci, 9 * Co).contiguous()     # [Cin][kh][kw][Cout] (flip: address mode)
        dx = K.conv3x3_bwd_data(dy, w_bwd)
        ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1)
        err = rel(dx.permute(0, 3, 1, 2), ref)
        ms = timed(lambda: K.conv3x3_bwd_data(dy, w_bwd))
        rows.append((f"conv bwd-data {Co}->{Ci} {H}x{W}", ms, fl, err))
    tot = 0.0
    for tag, ms, fl, err in rows:
        tot += ms
        print(f"{tag:32s} {ms * 1e3:9.1f} us  {fl / ms / 1e9:8.1f} TFLOP/s  rel.err {err:.2e}")
    print(f"total {tot:.3f} ms  (OCRK_GEMM_PP={os.environ.get('OCRK_GEMM_PP', '1')}, "
          "no vendor route)", flush=True)


if __name__ == "__main__":
    main()
