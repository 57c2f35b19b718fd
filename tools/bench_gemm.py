"""GEMM-engine microbenchmark on the train step's shapes (diagnostic).

    python tools/bench_gemm.py            # engine chosen by OCRK_GEMM_NT (default: NT engine on)
Prints one line per shape: ms per launch and TFLOP/s, and a checksum so two
runs (OCRK_GEMM_NT=0 / 1) can be compared for agreement.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

B = 256
CONV = [(30, 254, 32, 32), (15, 127, 32, 64), (15, 127, 64, 64), (7, 126, 64, 128), (7, 126, 128, 128),
        (3, 125, 128, 256), (3, 125, 256, 256)]


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        out = fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps, out


def main():
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    torch.manual_seed(0)
    dev = torch.device("cuda")
    bf = torch.bfloat16
    rows = []
    for (M, N, Kd, tag) in [(32000, 4096, 256, "proj L1"), (32000, 4096, 1024, "proj L2"),
                            (32000, 1024, 4096, "dx L2"), (32000, 256, 4096, "dx L1"),
                            (32000, 1024, 96, "logits dx"), (32000, 96, 1024, "logits fwd")]:
        if only and only not in tag:
            continue
        a = torch.randn(M, Kd, device=dev).to(bf)
        w = torch.randn(N, Kd, device=dev).to(bf) * 0.05
        bias = torch.randn(N, device=dev)
        ms, out = timed(lambda: K.gemm(a, w, trans_b=True, bias=bias, out_dtype=bf))
        rows.append((tag, ms, 2.0 * M * N * Kd, float(out.float().abs().sum())))
    for (H, W, Ci, Co) in ([] if only else CONV):
        x = torch.randn(B, H, W, Ci, device=dev).to(bf)
        w_nk = (torch.randn(Co, 9 * Ci, device=dev) * 0.05).to(bf)
        bias = torch.zeros(Co, device=dev)
        ms, out = timed(lambda: K.conv3x3_fwd(x, w_nk, bias, relu=True))
        fl = 2.0 * B * H * W * 9 * Ci * Co
        rows.append((f"conv fwd {Ci}->{Co} {H}x{W}", ms, fl, float(out.float().abs().sum())))
        dy = torch.randn(B, H, W, Co, device=dev).to(bf)
        w_bwd = (torch.randn(Ci, 9 * Co, device=dev) * 0.05).to(bf)
        ms, out = timed(lambda: K.conv3x3_bwd_data(dy, w_bwd))
        rows.append((f"conv bwd-data {Co}->{Ci} {H}x{W}", ms, fl, float(out.float().abs().sum())))
    for (H, W, Ci, Co) in ([] if only else CONV):
        x = torch.randn(B, H, W, Ci, device=dev).to(bf)
        dy = torch.randn(B, H, W, Co, device=dev).to(bf)
        dw = torch.zeros(9 * Ci, Co, device=dev)
        def wg():
            dw.zero_()
            K.conv3x3_bwd_weight(x, dy, dw)
            return dw
        ms, out = timed(wg)
        rows.append((f"conv wgrad {Ci}->{Co} {H}x{W}", ms, 2.0 * B * H * W * 9 * Ci * Co,
                     float(out.abs().sum())))
    R = 32000
    for (n_in, tag) in [(1024, "LSTM dW_x L2"), (512, "LSTM dW_h"), (256, "LSTM dW_x L1")]:
        if only and only not in tag:
            continue
        x = torch.randn(R, n_in, device=dev).to(bf)
        dG = torch.randn(R, 4096, device=dev).to(bf)
        gk = torch.zeros(n_in, 2048, device=dev)
        def dwg():
            gk.zero_()
            K.gemm(x, dG, trans_a=True, out=gk, accumulate=True, M=n_in, N=2048, K=R, lda=n_in, ldb=4096,
                   ldc=2048, splits=max(1, min(-(-512 // (-(-n_in // 128) * 16)), R // 2048)))
            return gk
        ms, out = timed(dwg)
        rows.append((tag, ms, 2.0 * n_in * 2048 * R, float(out.abs().sum())))
    tot = 0.0
    for tag, ms, fl, chk in rows:
        tot += ms
        print(f"{tag:32s} {ms * 1e3:9.1f} us  {fl / ms / 1e9:8.1f} TFLOP/s  checksum {chk:.6e}")
    print(f"total {tot:.3f} ms  (OCRK_GEMM_NT={os.environ.get('OCRK_GEMM_NT', '1')}, "
          f"OCRK_GEMM_TN={os.environ.get('OCRK_GEMM_TN', '1')})")


if __name__ == "__main__":
    main()
