"""CTC loss (+ gradient) kernel timing at the bench shape (diagnostic).

    python tools/bench_ctc.py        # T=125, B=256, C=96, labels of 2..19 symbols
    python tools/bench_ctc.py --long # T=600, labels of 100..200 symbols (S up to 401:
                                     # the R = 8 lattice instance)
Prints per-launch time with the gradient and loss-only, for the lattices in
LDS (default) and in the global workspace (OCRK_CTC_LDS=0)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
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


def main():
    long = "--long" in sys.argv
    T, B, C = (600, 256, 96) if long else (125, 256, 96)
    lo, hi = (100, 201) if long else (2, 20)
    rng = np.random.default_rng(0)
    dev = torch.device("cuda")
    logits = torch.from_numpy(np.maximum(rng.standard_normal((T, B, C)) * 3, 0).astype(np.float32)).to(dev)
    ln = rng.integers(lo, hi, B).astype(np.int32)
    lab = np.zeros((B, hi - 1), np.int32)
    for i in range(B):
        lab[i, :ln[i]] = rng.integers(0, C - 1, ln[i])
    lab, ln = torch.from_numpy(lab).to(dev), torch.from_numpy(ln).to(dev)
    seq = torch.full((B,), T, dtype=torch.int32, device=dev)
    for mode in ("1", "0"):
        os.environ["OCRK_CTC_LDS"] = mode
        g = timed(lambda: K.ctc_loss(logits, lab, ln, seq))
        n = timed(lambda: K.ctc_loss(logits, lab, ln, seq, need_grad=False))
        loss = K.ctc_loss(logits, lab, ln, seq)[0]
        print(f"OCRK_CTC_LDS={mode}: loss+grad {g:7.1f} us   loss only {n:7.1f} us   sum(loss) {loss.sum().item():.6e}")


if __name__ == "__main__":
    main()
