"""Micro-benchmark of the recurrent step kernels (diagnostics, not the product path)."""
import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# debug stamps (include/ocrk_debug.h) live in the tools-only build: `make exp`
os.environ.setdefault("OCRK_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libocrk_exp.so"))
from cnn_lstm_ctc_ocr_amd import kernels as K, _lib

def run(B, H=512, n_in=1024, T=125, reps=3, dt=torch.bfloat16):
    os.environ["OCRK_LSTM_PERSISTENT"] = "0"
    K._PERSISTENT.clear()
    dev = torch.device("cuda")
    gx = torch.randn(T * B, 8 * H, device=dev).to(dt)
    whT = (torch.randn(2, 4 * H, H, device=dev) * 0.02).to(dt)
    wh = (torch.randn(2, H, 4 * H, device=dev) * 0.02).to(dt)
    seq = torch.full((B,), T, dtype=torch.int32, device=dev)
    out, hprev, cprev, acts = K.lstm_fwd(gx, whT, seq, T, B, H, dt)
    dout = torch.randn(T, B, 2 * H, device=dev).to(dt)
    K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    for _ in range(reps):
        K.lstm_fwd(gx, whT, seq, T, B, H, dt)
    e[1].record()
    for _ in range(reps):
        K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H)
    e[2].record()
    torch.cuda.synchronize()
    f = e[0].elapsed_time(e[1]) / reps / T * 1e3
    b = e[1].elapsed_time(e[2]) / reps / T * 1e3
    print(f"B={B:4d} H={H}: fwd step {f:7.2f} us   bwd step {b:7.2f} us", flush=True)

for B in ([int(a) for a in sys.argv[1:] if a.isdigit()] or (64, 128, 256, 512)):
    run(B)

# in-kernel stamps of one forward step (thread 0 of each workgroup, 100 MHz clock)
if "--stamps" in sys.argv:
    import numpy as np
    B, H, T = 256, 512, 8
    dev = torch.device("cuda")
    dbg = torch.zeros(2 * 4 * 32 * 8, dtype=torch.int64, device=dev)
    gx = torch.randn(T * B, 8 * H, device=dev).bfloat16()
    whT = (torch.randn(2, 4 * H, H, device=dev) * 0.02).bfloat16()
    seq = torch.full((B,), T, dtype=torch.int32, device=dev)
    K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)
    torch.cuda.synchronize()
    _lib.call("ocrk_lstm_debug_stamps", _lib.ptr(dbg))
    K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)     # every launch overwrites: the last step remains
    torch.cuda.synchronize()
    _lib.call("ocrk_lstm_debug_stamps", None)
    st = dbg.view(-1, 8)[:, :6].cpu().numpy().astype(np.float64) * 10.0   # ns
    t0 = st[:, 0].min()
    print("stamp (ns since first WG start): median / max over workgroups")
    names = ["start", "gemm loads issued", "epilogue loads issued", "gemm done", "spill done", "end"]
    if os.environ.get("OCRK_LSTM_DMA", "1") != "0":
        names = ["start", "dma issued", "epilogue loads issued", "operands landed", "mfma+spill done", "end"]
    for i, n in enumerate(names):
        print(f"  {n:24s} {np.median(st[:, i] - t0):9.0f} {np.max(st[:, i] - t0):9.0f}")
    d = st[:, 1:] - st[:, :-1]
    for i in range(5):
        print(f"  {names[i]} -> {names[i+1]}: median {np.median(d[:, i]):8.0f} ns")

if "--persistent" in sys.argv:
    import numpy as np
    for B in (64, 256):
        H, T = 512, 125
        dev = torch.device("cuda")
        gx = torch.randn(T * B, 8 * H, device=dev).bfloat16()
        whT = (torch.randn(2, 4 * H, H, device=dev) * 0.05).bfloat16()
        seq = torch.randint(T // 2, T + 1, (B,), dtype=torch.int32, device=dev)
        os.environ["OCRK_LSTM_PERSISTENT"] = "0"
        K._PERSISTENT.clear()
        ref = K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)
        os.environ["OCRK_LSTM_PERSISTENT"] = "1"
        K._PERSISTENT.clear()
        print("persistent supported:", K.lstm_persistent_ok(B, H, torch.bfloat16))
        got = K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)
        torch.cuda.synchronize()
        print("err word:", K.lstm_error_word(dev).item())
        for name, a, b in zip(("out", "hprev", "cprev", "acts"), ref, got):
            d = (a.float() - b.float()).abs().max().item()
            print(f"  {name}: max |step-kernel - persistent| = {d:.3e}")
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        for _ in range(5):
            K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)
        e[1].record()
        torch.cuda.synchronize()
        print(f"B={B}: persistent fwd {e[0].elapsed_time(e[1]) / 5 / T * 1e3:.2f} us/step, err={K.lstm_error_word(dev).item()}")
        wh = (torch.randn(2, H, 4 * H, device=dev) * 0.05).bfloat16()
        dout = torch.randn(T, B, 2 * H, device=dev).bfloat16()
        _, _, cprev, acts = got
        os.environ["OCRK_LSTM_PERSISTENT"] = "0"
        K._PERSISTENT.clear()
        dref = K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H)
        e[0].record()
        for _ in range(5):
            K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H)
        e[1].record()
        torch.cuda.synchronize()
        print(f"B={B}: step-kernel bwd {e[0].elapsed_time(e[1]) / 5 / T * 1e3:.2f} us/step")
        os.environ["OCRK_LSTM_PERSISTENT"] = "1"
        K._PERSISTENT.clear()
        dgot = K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H)
        torch.cuda.synchronize()
        d = (dref.float() - dgot.float()).abs().max().item()
        print(f"  dG: max |step-kernel - persistent| = {d:.3e} (max |dG| {dref.float().abs().max().item():.3e})")
        e[0].record()
        for _ in range(5):
            K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H)
        e[1].record()
        torch.cuda.synchronize()
        print(f"B={B}: persistent bwd {e[0].elapsed_time(e[1]) / 5 / T * 1e3:.2f} us/step, err={K.lstm_error_word(dev).item()}")

if "--pstamps" in sys.argv:
    import numpy as np
    os.environ["OCRK_LSTM_PERSISTENT"] = "1"
    K._PERSISTENT.clear()
    B, H, T = 256, 512, 125
    dev = torch.device("cuda")
    gx = torch.randn(T * B, 8 * H, device=dev).bfloat16()
    whT = (torch.randn(2, 4 * H, H, device=dev) * 0.05).bfloat16()
    seq = torch.full((B,), T, dtype=torch.int32, device=dev)
    K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)
    dbg = torch.zeros(256 * 8, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    _lib.call("ocrk_lstm_debug_stamps", _lib.ptr(dbg))
    K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)
    torch.cuda.synchronize()
    _lib.call("ocrk_lstm_debug_stamps", None)
    st = dbg.view(-1, 8)[:, :7].cpu().numpy().astype(np.float64) * 10.0
    names = ["top", "poll done", "h+gx staged", "mfma+spill done", "cell+flag done", "outputs issued", "next top"]
    t0 = st[:, 0].min()
    for i, n in enumerate(names):
        print(f"  {n:16s} median {np.median(st[:, i] - t0):8.0f}  max {np.max(st[:, i] - t0):8.0f} ns")
    d = np.diff(st, axis=1)
    for i in range(6):
        print(f"  {names[i]:>14s} -> {names[i+1]:14s}: median {np.median(d[:, i]):7.0f} ns  max {np.max(d[:, i]):7.0f}")

if "--bstamps" in sys.argv:
    import numpy as np
    os.environ["OCRK_LSTM_PERSISTENT"] = "1"
    K._PERSISTENT.clear()
    B, H, T = 256, 512, 125
    dev = torch.device("cuda")
    gx = torch.randn(T * B, 8 * H, device=dev).bfloat16()
    whT = (torch.randn(2, 4 * H, H, device=dev) * 0.05).bfloat16()
    wh = (torch.randn(2, H, 4 * H, device=dev) * 0.05).bfloat16()
    seq = torch.full((B,), T, dtype=torch.int32, device=dev)
    _, _, cprev, acts = K.lstm_fwd(gx, whT, seq, T, B, H, torch.bfloat16)
    dout = torch.randn(T, B, 2 * H, device=dev).bfloat16()
    K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H)
    dbg = torch.zeros(256 * 8, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    _lib.call("ocrk_lstm_debug_stamps", _lib.ptr(dbg))
    K.lstm_bwd(wh, seq, dout, cprev, acts, T, B, H)
    torch.cuda.synchronize()
    _lib.call("ocrk_lstm_debug_stamps", None)
    st = dbg.view(-1, 8)[:, [0, 1, 2, 3, 4, 6]].cpu().numpy().astype(np.float64) * 10.0
    print("  workgroups with an XCD-local group:", int(dbg.view(-1, 8)[:, 7].sum().item()), "of 256")
    names = ["top", "poll done", "mfma+spill done", "cell+flag done", "dG issued", "next top"]
    t0 = st[:, 0].min()
    for i, n in enumerate(names):
        print(f"  {n:16s} median {np.median(st[:, i] - t0):8.0f}  max {np.max(st[:, i] - t0):8.0f} ns")
    d = np.diff(st, axis=1)
    for i in range(5):
        print(f"  {names[i]:>14s} -> {names[i+1]:14s}: median {np.median(d[:, i]):7.0f} ns  max {np.max(d[:, i]):7.0f}")
