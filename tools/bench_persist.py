"""Persistent recurrent loops alone (diagnostics): per-step time of the
persistent LSTM forward / BPTT at the bench shape, both BPTT forms, and the
in-kernel s_memrealtime stamps of one mid-sequence step.
    python tools/bench_persist.py [B] [H]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# debug stamps (include/ocrk_debug.h) live in the tools-only build: `make exp`
os.environ.setdefault("OCRK_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libocrk_exp.so"))
from cnn_lstm_ctc_ocr_amd import _lib, kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
H = int(sys.argv[2]) if len(sys.argv) > 2 else 512
T = 125
dev = torch.device("cuda")
torch.manual_seed(0)
gx = (torch.randn(T * B, 8 * H, device=dev) * 0.5).bfloat16()
whT = (torch.randn(2, 4 * H, H, device=dev) * 0.02).bfloat16()
wh = whT.transpose(1, 2).contiguous()
seq = torch.full((B,), T, dtype=torch.int32, device=dev)
out, hprev, cprev, acts = K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)
dout = (torch.randn(T, B, 2 * H, device=dev) * 0.1).bfloat16()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3 / T


os.environ["OCRK_PERSIST_LATE"] = "0"
f0 = timed(lambda: K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16))
os.environ["OCRK_LSTM_BWD_KSPLIT"] = "0"
b0 = timed(lambda: K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H))
ref_fwd = K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)[0].float()
ref_bwd = K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H).float()
os.environ["OCRK_PERSIST_LATE"] = "1"
f = timed(lambda: K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16))
late_fwd = K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)[0].float()
late_bwd = K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H).float()
torch.cuda.synchronize()
print(f"late loads: fwd {f0:.2f} -> {f:.2f} us/step (max diff {(late_fwd - ref_fwd).abs().max().item():.1e}); "
      f"gather bwd {b0:.2f} -> (below) (max diff {(late_bwd - ref_bwd).abs().max().item():.1e})", flush=True)
res, outs = {}, {}
for form, pb in (("1", "0"), ("1", "1"), ("0", "0")):
    os.environ["OCRK_LSTM_BWD_KSPLIT"], os.environ["OCRK_LSTM_BWD_PB16"] = form, pb
    res[form + pb] = timed(lambda: K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H))
    outs[form + pb] = K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H).float()
torch.cuda.synchronize()
os.environ["OCRK_LSTM_BWD_PB16"] = "0"
dg = outs["00"]
d = {k: ((v - dg).norm() / dg.norm()).item() for k, v in outs.items()}
print(f"B={B} H={H} T={T}: fwd {f:.2f} us/step; bwd K-split f32 {res['10']:.2f}, K-split bf16 {res['11']:.2f}, "
      f"gather {res['00']:.2f} us/step; rel diff vs gather: f32 {d['10']:.2e} bf16 {d['11']:.2e}; "
      f"status {K.read_status(dev)}", flush=True)

names = {"fwd": ["start", "flags seen", "h staged", "gates spilled", "h published", "saved stored"],
         "ksplit": ["start", "flags seen", "dz in LDS", "P published", "dG stored"],
         "gather": ["start", "flags seen", "partials met", "dz published", "dG stored"]}
for kind in ("fwd", "ksplit", "gather"):
    dbg = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
    os.environ["OCRK_LSTM_BWD_KSPLIT"] = "0" if kind == "gather" else "1"
    _lib.call("ocrk_lstm_debug_stamps", _lib.ptr(dbg))
    if kind == "fwd":
        K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)
    else:
        K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H)
    torch.cuda.synchronize()
    _lib.call("ocrk_lstm_debug_stamps", None)
    n = len(names[kind])
    grid = 2 * (B // 32) * (H // 32)
    st = dbg.view(-1, 8)[:grid].cpu().numpy().astype(np.float64) * 10.0          # 100 MHz -> ns
    top = st[:, 6]                                                               # top of the next step
    seg = [st[:, i] for i in range(n)] + [top]
    print(f"{kind}: step 64 -> 65 median {np.median(top - st[:, 0]):.0f} ns")
    for i in range(n):
        d = seg[i + 1] - seg[i]
        nxt = names[kind][i + 1] if i + 1 < n else "next step"
        print(f"  {names[kind][i]:>14s} -> {nxt:<14s} median {np.median(d):7.0f} ns  p90 {np.percentile(d, 90):7.0f}")
