"""Time the decoders on device-resident logits (diagnostic, not the bench line).

python tools/bench_decode.py [--B 256] [--T 63] [--beams 16,128]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cnn_lstm_ctc_ocr_amd import kernels as K


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--T", type=int, default=63)
    ap.add_argument("--beams", default="16,128")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    C = 96
    x = (rng.standard_normal((a.T, a.B, C)) * 0.5).astype(np.float32)
    cls = rng.integers(0, C, (a.T, a.B))
    cls[rng.random((a.T, a.B)) < 0.5] = C - 1
    np.put_along_axis(x, cls[..., None], 7.0, axis=2)
    dev = torch.device("cuda:0")
    logits = torch.from_numpy(x).to(dev)
    seq = torch.full((a.B,), a.T, dtype=torch.int32, device=dev)
    res = {}

    def timed(name, fn):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t) / a.reps * 1e3

    timed("greedy", lambda: K.ctc_greedy_decode(logits, seq))
    for k in map(int, a.beams.split(",")):
        timed(f"beam{k}", lambda k=k: K.ctc_beam_decode(logits, seq, k, 1, True))
    for kind in ("random",):
        xr = torch.from_numpy((rng.standard_normal((a.T, a.B, C)) * 2).astype(np.float32)).to(dev)
        for k in map(int, a.beams.split(",")):
            timed(f"beam{k}_{kind}", lambda k=k: K.ctc_beam_decode(xr, seq, k, 1, True))
    for n, ms in res.items():
        print(f"{n:16s} {ms:9.3f} ms  ({a.B / ms * 1e3:10.0f} seq/s)  B={a.B} T={a.T}")


if __name__ == "__main__":
    main()
