"""Vendor-library reference points on the train step's GEMM / conv shapes (diagnostic only).

    python tools/bench_vendor.py
torch.matmul (hipBLASLt) for the recurrent projections and F.conv2d (MIOpen,
channels-last bf16) for the conv tower: what the ROCm libraries reach on
these shapes, as a yardstick for the hand-written engines (bench_gemm.py).
Nothing here is on the product path.
"""
import torch
import torch.nn.functional as F

B = 256
CONV = [(30, 254, 32, 32), (15, 127, 32, 64), (15, 127, 64, 64), (7, 126, 64, 128), (7, 126, 128, 128),
        (3, 125, 128, 256), (3, 125, 256, 256)]


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda")
    bf = torch.bfloat16
    for (M, N, Kd, tag) in [(32000, 4096, 256, "proj L1"), (32000, 4096, 1024, "proj L2"),
                            (32000, 1024, 4096, "dx L2"), (32000, 256, 4096, "dx L1"),
                            (1024, 2048, 32000, "dW_x L2 (x^T dG)")]:
        if tag.startswith("dW"):
            a = torch.randn(32000, 1024, device=dev).to(bf).t()
            w = torch.randn(32000, 2048, device=dev).to(bf)
            ms = timed(lambda: a @ w)
        else:
            a = torch.randn(M, Kd, device=dev).to(bf)
            w = torch.randn(N, Kd, device=dev).to(bf)
            ms = timed(lambda: a @ w.t())
        print(f"hipBLASLt {tag:20s} {ms * 1e3:8.1f} us {2.0 * M * N * Kd / ms / 1e9:8.1f} TFLOP/s", flush=True)
    for (H, W, Ci, Co) in CONV:
        x = torch.randn(B, Ci, H, W, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
        w = torch.randn(Co, Ci, 3, 3, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
        try:
            ms = timed(lambda: F.conv2d(x, w, padding=1))
            fl = 2.0 * B * H * W * 9 * Ci * Co
            print(f"MIOpen conv fwd {Ci}->{Co} {H}x{W}: {ms * 1e3:8.1f} us {fl / ms / 1e9:8.1f} TFLOP/s", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"MIOpen conv fwd {Ci}->{Co}: {type(e).__name__}: {e}"[:200], flush=True)


if __name__ == "__main__":
    main()
