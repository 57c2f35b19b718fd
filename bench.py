#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): line-crops/sec per TRAIN STEP at
32x256, batch 256 per GPU, CNN -> BiLSTM(512, 512) -> CTC (src/weinman/model_bu.py),
bf16 compute, Adam update included -- configs[2] "Batch=256 synthetic 32x256
training step (conv+BiLSTM+CTC grad), 1xMI355X bf16"; with --gpus N the same
per-GPU batch runs data-parallel (weak scaling, one RCCL all-reduce per step).

One step = convnet_layers -> rnn_layers -> ctc_loss_layer forward, backward,
gradient all-reduce (N > 1) and the Adam kernel, on synthetic uint8 crops and
labels already resident in HBM. Rank 0 prints ONE JSON line.
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip table)
PEAK_F32_TFLOPS = 157.3       # f32 MFMA = f32 vector peak
# fp32 GEMMs run as the bf16x3 split (3 bf16 MFMA products per fp32 product,
# csrc/mfma_util.h): their roofline is the bf16 dense peak / 3
PEAK_F32X3_TFLOPS = PEAK_BF16_TFLOPS / 3
PEAK_HBM_GBS = 8000.0         # HBM3E spec


def synthetic_batch(rng, B, W, T, device):
    """uint8 crops U{0..255}; labels: length U{2..19}, chars U{0..94}, resampled
    until L + #repeats <= T."""
    img = torch.from_numpy(rng.integers(0, 256, (B, 32, W, 1), dtype=np.uint8)).to(device)
    widths = torch.full((B,), W, dtype=torch.int32, device=device)
    lab = np.zeros((B, 19), np.int32)
    ln = np.zeros(B, np.int32)
    for b in range(B):
        while True:
            L = int(rng.integers(2, 20))
            s = rng.integers(0, 95, L)
            if L + int(np.sum(s[1:] == s[:-1])) <= T:
                break
        lab[b, :L] = s
        ln[b] = L
    return img, widths, (torch.from_numpy(lab).to(device), torch.from_numpy(ln).to(device))


def work_conv_fwd(args):
    # (x, B, H, W, cin, w_nk, bias, cout, ...): 2 * pixels * 9 * cin * cout FLOP
    # (ocrk_conv3x3_fwd, _rowstats, _relu_bits)
    return 2.0 * args[1] * args[2] * args[3] * 9 * args[4] * args[7]


def work_conv12_fwd(args):
    # (x, x_is_u8, B, IH, IW, ...): conv1 (1 -> 32, 'valid') and conv2 (32 -> 32) over the
    # same B x (IH-2) x (IW-2) pixels in one launch
    return 2.0 * args[2] * (args[3] - 2) * (args[4] - 2) * 9 * (1 * 32 + 32 * 32)


def work_lstm_fwd(args):
    # (gx, whT, h, c, seq_len, T, B, H, ...): recurrent h.W_h FLOP, both directions
    T, B, H = args[5], args[6], args[7]
    return 2.0 * 2 * T * B * H * 4 * H


def work_gemm(args):
    # (ta, tb, M, N, K, ...., batch at index 19)
    return 2.0 * args[2] * args[3] * args[4] * args[19]


def work_dw(args):
    # the recurrent weight gradients dW = x^T dG, h_prev^T dG (trans_a, M, N >= 256:
    # gemm_pptn_kernel<A_COLK>, the step's largest kernel class); None filters the
    # other ocrk_gemm launches out of the probe
    if args[0] != 1 or args[2] < 256 or args[3] < 256:
        return None
    return work_gemm(args)


ROOFLINE_OPS = {
    # conv2-conv5 run on the row-walking kernels (ocrk_conv3x3_fwd_rowstats for the BN layers)
    "conv": (("ocrk_conv12_fwd", "ocrk_conv3x3_fwd", "ocrk_conv3x3_fwd_rowstats", "ocrk_conv3x3_fwd_relu_bits"),
             {"ocrk_conv12_fwd": work_conv12_fwd, "ocrk_conv3x3_fwd": work_conv_fwd,
              "ocrk_conv3x3_fwd_rowstats": work_conv_fwd, "ocrk_conv3x3_fwd_relu_bits": work_conv_fwd},
             "conv1-conv8 forward launches (conv1 -> conv2 as one row walk, row-walking conv3-conv5, implicit "
             "GEMM conv6-conv8; MFMA bf16)"),
    "lstm": ("ocrk_lstm_fwd", work_lstm_fwd, "recurrent h.W_h time loop, both directions (MFMA bf16)"),
    "gemm": ("ocrk_gemm", work_gemm, "dense GEMM launches"),
    "dw": ("ocrk_gemm", work_dw, "recurrent weight-gradient GEMMs dW = [x, h_prev]^T dG, both directions batched "
           "(gemm_pptn_kernel<A_COLK>, side stream; MFMA bf16)"),
}


def host_cpu():
    """(host threads for the CPU legs, CPU model name). The GPU box is a slice
    of a 256-CPU host whose CPU share is OMP_NUM_THREADS (16): more threads
    than that measured slower (16 / 32 / 64 threads: 35 / 23 / 8 crops/s on a
    16-crop train step), so the share is used when it is set."""
    try:
        threads = len(os.sched_getaffinity(0))
    except AttributeError:
        threads = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        threads = min(threads, int(share))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return threads, model


def _cpu_batch(rng, B, W):
    T = (W - 2) // 2 - 2
    img, _, (lab, ln) = synthetic_batch(rng, B, W, T, torch.device("cpu"))
    return img, lab.long(), ln.long()


RNN_SIZES = {"lstm": (512, 512), "gru": (512, 256)}     # model_bu.py (bench default) / model.py


def cpu_baseline(sample, warmup=3, steps=6, cell="lstm"):
    """BASELINE.md CPU-baseline plan: the reference graph's train step (conv ->
    BiLSTM 512/512 -> CTC -> TF1 Adam) as the PyTorch-CPU restatement
    (oracle/torch_ref.py, checked against the NumPy oracle in
    tests/test_oracle.py; TensorFlow 1.x is unavailable), with every host
    thread this process may use, on `sample` synthetic 32x256 crops -- by
    default the GPU step's own shape (B = 256), 3 warm-up + 6 timed steps
    (~30 s of host time, bounded so the default run stays within minutes); the
    per-step times' spread is reported beside the mean rate."""
    from oracle import ref_model as M
    from oracle.torch_ref import TorchRef
    threads, model = host_cpu()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        sizes = RNN_SIZES[cell]
        ref = TorchRef(M.init_params(seed=0, cell=cell, rnn_sizes=sizes), sizes, cell=cell)
        img, lab, ln = _cpu_batch(np.random.default_rng(20260), sample, 256)
        for _ in range(warmup):
            ref.train_step(img, lab, ln)
        print(f"# cpu baseline: {warmup} warm-up steps done", file=sys.stderr, flush=True)
        per = []
        for i in range(steps):
            t0 = time.perf_counter()
            ref.train_step(img, lab, ln)
            per.append(time.perf_counter() - t0)
            print(f"# cpu baseline: step {i + 1}/{steps}", file=sys.stderr, flush=True)
        dt = sum(per)
    finally:
        torch.set_num_threads(prev)
    rates = sorted(sample / t for t in per)
    return {"value": round(sample * steps / dt, 3), "unit": "line-crops/sec", "cores": threads, "kind": "port",
            "cpu": model, "per_step_s": [round(t, 3) for t in per],
            "spread": {"min": round(rates[0], 3), "median": round(float(np.median(rates)), 3),
                       "max": round(rates[-1], 3), "cv": round(float(np.std(per) / np.mean(per)), 4)},
            "sample": f"reference graph on CPU (PyTorch restatement oracle/torch_ref.py; TF1 unavailable): "
                      f"{warmup} warm-up + {steps} timed train steps (fp32, {cell.upper()} {sizes[0]}/{sizes[1]}, Adam) on {sample} "
                      f"synthetic 32x256 crops, {threads} threads, {dt:.1f} s"}


def c1_latency(device, reps=20):
    """BASELINE configs[0] (C1): one 32x128 crop, INFER forward + greedy decode
    (validate.py:131-177 with common.py's bucket_size=1): the CPU reference
    path (PyTorch restatement, all host threads) and this path on one GPU
    (fp32, the reference's precision), median latency."""
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, model, validate
    from oracle import ref_model as M
    from oracle.torch_ref import TorchRef
    rng = np.random.default_rng(20260)
    img = rng.integers(0, 256, (1, 32, 128, 1), dtype=np.uint8)
    threads, cpu = host_cpu()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        ref = TorchRef(M.init_params(seed=0), (512, 512))
        x = torch.from_numpy(img)
        cpu_ms = []
        for i in range(3 + reps):
            t0 = time.perf_counter()
            cpu_dec = ref.greedy(x)
            if i >= 3:
                cpu_ms.append(1e3 * (time.perf_counter() - t0))
    finally:
        torch.set_num_threads(prev)
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=torch.float32), device=device, seed=0)
    xd = torch.from_numpy(img).to(device)
    wd = torch.tensor([128], dtype=torch.int32)
    gpu_ms = []
    for i in range(3 + reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.no_grad():
            feats, seq = model.convnet_layers(xd, wd, model.INFER, store)
            dense = validate._get_output(model.rnn_layers(feats, seq, 95, store), seq)[0].cpu()
        if i >= 3:
            gpu_ms.append(1e3 * (time.perf_counter() - t0))
    same = [int(v) for v in dense[0].tolist() if v >= 0] == cpu_dec[0]
    # the same request through the serving path's captured graph (infer.InferGraph):
    # host crop -> static buffers, one graph launch, the decode read back
    from cnn_lstm_ctc_ocr_amd.infer import InferGraph
    g = InferGraph(store, batch=1, width=128, n_classes=95)
    xh, wh = torch.from_numpy(img), torch.tensor([128], dtype=torch.int32)
    graph_ms = []
    for i in range(3 + reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.run(xh, wh)
        gdec = g.decoded.cpu()
        if i >= 3:
            graph_ms.append(1e3 * (time.perf_counter() - t0))
    same_graph = [int(v) for v in gdec[0].tolist() if v >= 0] == cpu_dec[0]
    return {"workload": "C1: 1 crop 32x128, INFER forward + greedy decode, reference initialisers",
            "cpu_ms": round(float(np.median(cpu_ms)), 3), "cpu_threads": threads, "cpu": cpu,
            "gpu_ms": round(float(np.median(gpu_ms)), 3), "gpu_dtype": "f32",
            "gpu_note": "host wall time incl. launches and the decode's device->host copy",
            "gpu_graph_ms": round(float(np.median(graph_ms)), 3),
            "gpu_graph_note": "the same request as one replay of the captured forward (infer.InferGraph), "
                              "host crop copied in, decode read back",
            "decode_equal": bool(same and same_graph)}


def cer_vs_ref(device):
    """The "CER vs ref" half of BASELINE.json's metric, measured outside the
    timed region: the HIP path's greedy (validate.py:81-92) and beam-16
    (test.py:84-88 with BASELINE configs[4]'s width) decodes of the committed
    golden batch (tests/golden/mjsynth_test_bucket.npz: 8 real crops of the
    reference's data/test shard, serving uint8 layout and training float
    layout) against the float64 oracle's decodes stored in that fixture, with
    the reference initialisers (seed 0, LSTM 512/512; no trained checkpoint
    exists). CER = sum(edit distance) / sum(len(oracle decode)) (test.py:90-99,
    tf.edit_distance normalize=False), on device; fp32 and bf16 compute."""
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, decode, model
    g = np.load(os.path.join(ROOT, "tests", "golden", "mjsynth_test_bucket.npz"))
    widths = torch.from_numpy(g["widths"])
    res = {"data": "tests/golden/mjsynth_test_bucket.npz (8 crops, data/test shard), oracle decodes at seed-0 weights"}
    for dname, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=dt), device=device, seed=0)
        edits = {"greedy": [0, 0, 0], "beam16": [0, 0, 0]}         # sum edit, sum ref length, rows differing
        for inp in ("u8", "f32"):
            x = torch.from_numpy(g["x_u8"] if inp == "u8" else g["x_f32"]).to(device)
            if inp == "f32":
                x = x.to(dt)
            with torch.no_grad():
                feats, seq = model.convnet_layers(x, widths, model.INFER, store)
                logits = model.rnn_layers(feats, seq, 95, store).float()
                hyps = {"greedy": decode.ctc_greedy_decoder(logits, seq)[0][0],
                        "beam16": decode.ctc_beam_search_decoder(logits, seq, beam_width=16)[0][0]}
            for kind, hyp in hyps.items():
                ref = torch.from_numpy(g[f"{inp}_{kind}"]).to(device)
                ref_len = (ref >= 0).sum(1).to(torch.int32)
                hyp_len = (hyp >= 0).sum(1).to(torch.int32)
                d = decode.edit_distance(hyp, hyp_len, ref.to(torch.int32), ref_len).cpu().numpy()
                edits[kind][0] += float(d.sum())
                edits[kind][1] += int(ref_len.sum().item())
                edits[kind][2] += int((d > 0).sum())
        for kind, (e, n, rows) in edits.items():
            res[f"{dname}_{kind}"] = {"cer": round(e / max(n, 1), 5), "rows_differing": rows, "rows": 16}
    return res


def cer_vs_ref_trained(device):
    """"CER vs ref" at TRAINED weights, outside the timed
    region: the LSTM 512/512 model trained in fp32 on the reference's data/val
    shard (tests/trained_model.py REGIME: 4,000 Trainer.steps, ~20 s), then every
    crop of the held-out data/test shard (892) through server.Bucket's 32-px uint8
    buckets, greedy and beam-16. The reference strings are the fp32 HIP path's --
    equal to the float64 reference graph's on all 932 served rows at these
    weights but one beam near-tie (tests/test_gpu_trained_serving.py,
    profiles/r6d_trained.json); the benched precision (bf16, the same weights)
    is scored against them: CER = sum(edit distance) / sum(len(reference
    string)) (test.py:90-99). Plus the fp32 model's greedy CER against the shard's
    own labels (generalisation from 800 training crops: context, not parity)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import trained_model as TM
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, decode, model
    t0 = time.perf_counter()
    store, _losses, _c = TM.train_on_shard(torch.float32, TM.shard_batches(TM.TRAIN_SHARD), device)
    train_s = time.perf_counter() - t0
    print(f"# trained CER: fp32 model trained in {train_s:.1f} s", file=sys.stderr, flush=True)
    bf = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=torch.bfloat16), device=device,
                    values=store.state_dict())
    tally = {k: [0, 0, 0] for k in ("greedy", "beam16")}      # sum edit, sum ref length, rows differing
    truth = [0, 0]
    rows = 0
    for _name, batch, widths, labels in TM.bucketed(TM.rows32(TM.shard_items(TM.HELD_OUT_SHARD))):
        x = torch.from_numpy(batch).to(device)
        w = torch.from_numpy(widths).to(device)
        out = {}
        with torch.no_grad():
            for tag, st in (("ref", store), ("bf16", bf)):
                feats, seq = model.convnet_layers(x, w, model.INFER, st)
                logits = model.rnn_layers(feats, seq, 95, st).float()
                out[tag] = {"greedy": decode.ctc_greedy_decoder(logits, seq)[0][0],
                            "beam16": decode.ctc_beam_search_decoder(logits, seq, beam_width=16)[0][0]}
        for kind in tally:
            ref, hyp = out["ref"][kind], out["bf16"][kind]
            ref_len, hyp_len = (ref >= 0).sum(1).to(torch.int32), (hyp >= 0).sum(1).to(torch.int32)
            d = decode.edit_distance(hyp, hyp_len, ref.to(torch.int32), ref_len).cpu().numpy()
            tally[kind][0] += float(d.sum())
            tally[kind][1] += int(ref_len.sum().item())
            tally[kind][2] += int((d > 0).sum())
        lab, ln = model.dense_labels(labels, len(labels), device)
        g = out["ref"]["greedy"]
        d = decode.edit_distance(g, (g >= 0).sum(1).to(torch.int32), lab, ln).cpu().numpy()
        truth[0] += float(d.sum())
        truth[1] += int(ln.sum().item())
        rows += len(labels)
    res = {"data": f"tests/golden/mjsynth_test_words000.npz (data/test shard, {rows} crops, server buckets, uint8); "
                   "weights: fp32 training on data/val (tests/trained_model.py REGIME, "
                   f"{TM.REGIME['steps']} steps, {train_s:.0f} s)",
           "reference": "the fp32 HIP path's strings (= the float64 graph's on all 932 served rows but one beam "
                        "near-tie: tests/test_gpu_trained_serving.py)",
           "fp32_greedy_cer_vs_labels": round(truth[0] / max(truth[1], 1), 4)}
    for kind, (e, n, diff) in tally.items():
        res[f"bf16_{kind}"] = {"cer": round(e / max(n, 1), 5), "rows_differing": diff, "rows": rows}
    return res


def run_c2(args, world, rank, device):
    """BASELINE configs[1] (C2): B=64 synthetic 32x256 crops, INFER forward +
    CTC loss + greedy decode, fp32 (test.py:75-104's evaluation graph with the
    greedy decoder of validate.py:81-92). One line, value = crops/s."""
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, decode, model
    B, W = 64, 256
    T = (W - 2) // 2 - 2
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=torch.float32), device=device, seed=0)
    img, widths, labels = synthetic_batch(np.random.default_rng(1234 + rank), B, W, T, device)

    def step():
        # the decode stays on the device (ctc_greedy_decoder_raw: [B, T] labels then -1):
        # validate._get_output's host read of the longest decode (its dense width) would
        # serialise every batch's launches behind the previous batch's kernels
        with torch.no_grad():
            feats, seq = model.convnet_layers(img, widths, model.INFER, store)
            logits = model.rnn_layers(feats, seq, 95, store)
            loss = model.ctc_loss_layer(logits, labels, seq, check=False)
            dense = decode.ctc_greedy_decoder_raw(logits, seq)[0]
        return loss, dense
    if args.c2_mode == "graph":
        # the same launches captured once (infer.InferGraph on the resident batch) and
        # replayed: one graph launch per batch instead of the Python walk over ~45 ops
        from cnn_lstm_ctc_ocr_amd.infer import InferGraph
        g = InferGraph(store, image=img, widths=widths, labels=labels, n_classes=95)

        def step():   # noqa: F811
            g.replay()
            return g.loss, g.decoded
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, _ = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return {"metric": "line-crops/sec (fwd + CTC loss + greedy decode) at 32x256 bs=64",
            "value": round(world * B * args.steps / elapsed, 2), "unit": "line-crops/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (uint8 crops, labels len U{2..19}; reference initialisers)",
            "config": {"workload": "C2: INFER fwd + CTC loss + greedy, LSTM 512/512", "per_gpu_batch": B,
                       "decode_output": "device [B, T] dense (-1 padded), read back after the timed steps",
                       "execution": "hipGraph replay per batch (infer.InferGraph)" if args.c2_mode == "graph"
                       else "eager launches",
                       "image": f"32x{W}", "parallelism": f"dp{world}",
                       "hip_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "HIP default (4)")},
            "loss": round(float(loss.item()), 4)}, elapsed, world * B * args.steps


def c5_buckets(n_crops=2048, seed=20265):
    """BASELINE configs[4] (C5) workload on the host: `n_crops` uint8 crops of
    true width U{65..512}, batched by the serving path's 32-px width buckets
    (server.py:28-42,64-65: bucket (w, w+32], crops right-padded with uint8 0 to
    its upper width). Returns [(upper width, images u8 [n, 32, upper, 1], true
    widths i32 [n])], largest bucket first. tests/test_gpu_configs.py checks
    this exact workload against the masked float64 graph."""
    rng = np.random.default_rng(seed)
    true_w = rng.integers(65, 513, n_crops)
    upper = ((true_w - 1) // 32 + 1) * 32                       # bucket (w, w + 32] -> its upper width
    buckets = sorted({int(u) for u in upper}, key=lambda u: -int((upper == u).sum()))
    out = []
    for u in buckets:
        idx = np.nonzero(upper == u)[0]
        img = np.zeros((len(idx), 32, u, 1), np.uint8)
        for j, i in enumerate(idx):
            img[j, :, :true_w[i]] = rng.integers(0, 256, (32, true_w[i], 1))
        out.append((u, img, true_w[idx].astype(np.int32)))
    return out


def run_c5(args, world, rank, device, n_crops=2048, beam=16):
    """BASELINE configs[4] (C5): c5_buckets' variable-width crops, INFER
    forward + beam-16 decode per bucket, fp32. Whole buckets are sharded over
    the ranks (largest first, round robin) -- replicas, no exchange (SURVEY
    8e). value = crops/s of the whole job."""
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, decode, model
    allb = c5_buckets(n_crops)
    buckets = [u for u, _, _ in allb]
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=torch.float32), device=device, seed=0)
    batches = [(torch.from_numpy(img).to(device), torch.from_numpy(w))
               for i, (_u, img, w) in enumerate(allb) if i % world == rank]

    # the beam search of bucket i runs on a second stream, beside the forward of
    # bucket i + 1 (it is latency-bound on ~B/4 workgroups: one wave per sequence)
    dec_stream = torch.cuda.Stream(device) if args.c5_pipeline else None

    graphs = None
    if args.c5_mode == "graph":
        # one captured INFER forward per bucket shape (infer.InferGraph on the resident
        # bucket), the beam search launched eagerly beside it
        from cnn_lstm_ctc_ocr_amd.infer import InferGraph
        graphs = [InferGraph(store, image=img, widths=w.to(device), decoder=None, n_classes=95)
                  for img, w in batches]

    def forward(i):
        if graphs is not None:
            g = graphs[i].replay()
            return g.logits, g.seq_len
        img, w = batches[i]
        feats, seq = model.convnet_layers(img, w, model.INFER, store)
        return model.rnn_layers(feats, seq, 95, store), seq

    def run():
        out = []
        main = torch.cuda.current_stream(device)
        for i in range(len(batches)):
            with torch.no_grad():
                logits, seq = forward(i)
                if dec_stream is None:
                    out.append(decode.ctc_beam_search_decoder_raw(logits, seq, beam_width=beam))
                    continue
                dec_stream.wait_stream(main)
                with torch.cuda.stream(dec_stream):
                    out.append(decode.ctc_beam_search_decoder_raw(logits, seq, beam_width=beam))
                logits.record_stream(dec_stream)
                seq.record_stream(dec_stream)
        if dec_stream is not None:
            main.wait_stream(dec_stream)
        return out
    for _ in range(max(1, args.warmup // 2)):
        run()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = max(1, args.steps // 4)
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = (time.perf_counter() - t0) / reps
    return {"metric": "line-crops/sec (bucketed 32x{64..512}, INFER + beam-16 decode)",
            "value": round(n_crops / elapsed, 2), "unit": "line-crops/sec", "n_gpus": world, "steps": reps,
            "warmup": max(1, args.warmup // 2), "ms_per_step": round(1e3 * elapsed, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic: {n_crops} uint8 crops, true widths U{{65..512}}, server-style 32-px buckets",
            "config": {"workload": "C5: bucketed INFER + CTC beam search (beam 16), LSTM 512/512",
                       "buckets": len(buckets), "crops": n_crops, "beam_width": beam,
                       "hip_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "HIP default (4)"),
                       "parallelism": f"replicas x{world} (whole buckets per rank)",
                       "decode": "second stream, beside the next bucket's forward" if args.c5_pipeline
                       else "in line",
                       "execution": "hipGraph replay of each bucket's forward (infer.InferGraph)"
                       if args.c5_mode == "graph" else "eager launches"}}, elapsed, n_crops


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, timeout=None):
    """`bench.py --gpus N` (N > 1) started WITHOUT a launcher (no WORLD_SIZE in
    the environment): start N fresh child processes of this script, one per
    GPU, BEFORE anything here touches the GPU (this parent never initialises
    HIP). Each child gets RANK = LOCAL_RANK = r, WORLD_SIZE = N and a
    127.0.0.1 rendezvous, binds cuda:LOCAL_RANK and joins the process group
    (RCCL; gloo in --selftest). Rank 0 prints the one aggregated JSON line on
    the inherited stdout. If a rank fails, the others are terminated (they
    would block in the next collective) and the parent exits non-zero.
    SURVEY 8e / DESIGN 7: one process per GPU, no exchange beyond the
    gradient all-reduce."""
    import threading
    port = _free_port()
    procs, pumps = [], []

    def pump(rank, pipe):
        # stdout carries exactly one line: rank 0's JSON result; library chatter
        # (gloo / RCCL banners) and every other rank's output go to stderr
        for line in iter(pipe.readline, ""):
            out = sys.stdout if (rank == 0 and line.lstrip().startswith("{")) else sys.stderr
            out.write(line)
            out.flush()
        pipe.close()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                             stdout=subprocess.PIPE, text=True, bufsize=1)
        procs.append(p)
        pumps.append(threading.Thread(target=pump, args=(r, p.stdout), daemon=True))
        pumps[-1].start()
    t0 = time.time()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"# bench launcher: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        if timeout is not None and time.time() - t0 > timeout and live:
            print("# bench launcher: timeout; stopping the ranks", file=sys.stderr, flush=True)
            for q in live:
                q.kill()
            rc = rc or 124
        time.sleep(0.05)
    for t in pumps:
        t.join(timeout=10)
    return rc


def _stand_in_grad(rng_seed, n):
    """A rank's stand-in gradient: a fixed function of its seed (every rank can
    recompute every other rank's)."""
    return torch.from_numpy(np.random.default_rng(rng_seed).standard_normal(n).astype(np.float32))


def selftest(args, world, rank):
    """--selftest: the C4 data-parallel protocol of this script on the CPU
    under gloo (no GPU): the launch, then per step the C4 partition -- each
    rank draws its own `--batch` crops from seed base + rank exactly as the GPU
    step does (synthetic_batch) -- the gradient exchange of train.GradBuckets
    over the real LSTM 512/512 ParamStore layout (the recurrent + logits bucket
    started from the mid-backward hook, then the conv bucket), the device
    status word OR-reduced over the ranks, and the barrier / max-over-ranks
    timing / one-line protocol. The forward + backward is a stand-in (a
    gradient that is a fixed function of the rank's batch), so the exchange is
    checked exactly: every rank must hold the sum of all ranks' gradients and
    the OR of their status bits (tests/test_bench_launcher.py). It is not a
    benchmark and its line says so."""
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import GradBuckets, or_allreduce_status
    if world > 1:
        dist.init_process_group("gloo")
    B, W = args.batch, args.width
    T = (W - 2) // 2 - 2
    store = ParamStore(ModelConfig(cell=args.cell, rnn_sizes=RNN_SIZES[args.cell], dtype=torch.float32),
                       device="cpu", seed=0)
    buckets = GradBuckets(store)
    n = store.flat_grad.numel()
    checks = {"partition": True, "allreduce": True, "status_or": True}
    seen = []

    def step(i):
        rng = np.random.default_rng(1234 + rank)                 # per-rank seed = base + rank (the GPU step's)
        img, widths, (lab, ln) = synthetic_batch(rng, B, W, T, "cpu")
        digest = int(img[:, 0, :8, 0].to(torch.int64).sum()) + int(ln.sum())
        seen.append(digest)
        g = store.flat_grad
        g.copy_(_stand_in_grad(1234 + rank + 7919 * i, n))     # the stand-in backward's gradient
        buckets.rnn_ready()                                      # the hook: recurrent + logits bucket
        scale = buckets.finish() if world > 1 else 1.0           # conv bucket, then wait for both
        word = torch.tensor([1 << (1 + rank % 6)], dtype=torch.int32)
        if world > 1:
            or_allreduce_status(word)
        return scale, word, digest
    for i in range(args.warmup):
        step(args.steps + i)                                     # its own stand-in gradients
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        scale, word, digest = step(i)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # exactness: the reduced gradient of the last step is the sum over ranks, the word the OR of their bits
    want = sum(_stand_in_grad(1234 + r + 7919 * (args.steps - 1), n).double() for r in range(world))
    checks["allreduce"] = bool(torch.allclose(store.flat_grad.double(), want, rtol=1e-5, atol=1e-5)) and \
        abs(scale - 1.0 / world) < 1e-12
    checks["status_or"] = int(word[0]) == int(np.bitwise_or.reduce([1 << (1 + r % 6) for r in range(world)]))
    ranks_seen = world
    digests = [digest]
    if world > 1:
        t = torch.tensor([elapsed, 1.0], dtype=torch.float64)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, ranks_seen = float(t[0]), int(t[1])
        gathered = [None] * world
        dist.all_gather_object(gathered, digest)
        digests = gathered
        ok = torch.tensor([int(all(checks.values()))], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        checks = {k: bool(v) and bool(ok[0]) for k, v in checks.items()}
    # C4's partition: distinct batches per rank, each the one its seed gives
    checks["partition"] = len(set(digests)) == world and len(set(seen)) == 1
    if rank == 0:
        print(json.dumps({"metric": "launcher self-test (CPU stand-in step, not a benchmark)",
                          "value": round(world * B * args.steps / elapsed, 2), "unit": "items/sec",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(1e3 * elapsed / args.steps, 3), "world_size_seen": ranks_seen,
                          "backend": "gloo", "checks": checks, "grad_values": n,
                          "config": {"global_batch": B * world, "per_gpu_batch": B,
                                     "parallelism": f"dp{world}", "seeds": f"1234 + rank (0..{world - 1})"}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="crops per GPU")
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--roofline", default="conv", choices=sorted(ROOFLINE_OPS))
    ap.add_argument("--roofline-also", default="dw",
                    help="comma-separated further roofline kinds reported in roofline_also (same timed steps)")
    ap.add_argument("--c5-mode", default="eager", choices=["graph", "eager"],
                    help="C5: each bucket's INFER forward launched eagerly (default) or replayed as a captured "
                         "HIP graph (measured slower: 22.5k vs 32.3k crops/s, profiles/r4_ab3.txt)")
    ap.add_argument("--c2-mode", default="graph", choices=["graph", "eager"],
                    help="C2: the INFER forward + loss + greedy decode replayed as one captured HIP graph "
                         "per batch (default), or launched eagerly")
    ap.add_argument("--mode", default="eager", choices=["graph", "eager"],
                    help="graph: forward+backward captured once as a HIP graph and replayed per step "
                         "(all-reduce + Adam eager); eager: every launch issued from Python each step")
    ap.add_argument("--breakdown", action="store_true", help="per-entry-point event timing table on stderr")
    ap.add_argument("--probe-every", type=int, default=4,
                    help="eager mode: the roofline kernel's HIP-event probes bracket its launches in every "
                         "Nth timed step (each probe event costs ~6 us of queue idle; 1 = every step)")
    ap.add_argument("--cpu-sample", type=int, default=256,
                    help="crops per CPU-baseline train step (default: the GPU step's B = 256)")
    ap.add_argument("--cpu-steps", type=int, default=6, help="timed CPU-baseline train steps (after 3 warm-up)")
    ap.add_argument("--config", default="c3", choices=["c3", "c2", "c5"],
                    help="c3: the headline train step (default); c2: B=64 fp32 fwd+CTC+greedy; "
                         "c5: bucketed 32x{64..512} crops, beam-16 decode")
    ap.add_argument("--c5-pipeline", type=int, default=1,
                    help="c5: 1 = each bucket's beam search on a second stream beside the next bucket's forward")
    ap.add_argument("--cell", default="lstm", choices=["lstm", "gru"],
                    help="lstm: model_bu.py's BiLSTM 512/512 (BASELINE.json's config); gru: model.py's BiGRU 512/256")
    ap.add_argument("--sync-bn", action="store_true",
                    help="C3 with N > 1: BatchNorm statistics over all ranks' batches (Trainer(sync_bn=True))")
    ap.add_argument("--main-stream", choices=("default", "own"), default="default",
                    help="run the train step on torch's default (NULL) stream or on a non-blocking stream of its own")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cer", action="store_true", help="skip the CER-vs-oracle decode check (outside the timing)")
    ap.add_argument("--no-trained-cer", action="store_true",
                    help="skip the trained-weight CER leg (~25 s: trains the model on data/val first)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_conv.json"),
                    help="PMC summary (tools/pmc_traffic.py) for roofline.traffic of the conv roofline kernel")
    ap.add_argument("--selftest", action="store_true",
                    help="CPU/gloo check of the multi-rank launch protocol with a stand-in step (no GPU)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start one process per GPU here, before any GPU call
        if not args.selftest and torch.cuda.device_count() < args.gpus:   # device_count does not initialise HIP
            sys.exit(f"bench.py --gpus {args.gpus}: only {torch.cuda.device_count()} GPUs visible")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.selftest:
        return selftest(args, world, rank)
    # HIP hardware queues per process, read once when HIP initialises (so here, before
    # the first HIP call): one process per GPU (world 1) running eager launches spreads
    # the step's streams (main, weight-gradient side stream, status copy) over 2
    # hardware queues -- 4.799-4.813 vs 4.821-4.828 ms/step with HIP's default 4, 3 and
    # 8 no better (profiles/r6_queues_ab.txt). OCRK_HW_QUEUES picks another count (the
    # GPU boxes export GPU_MAX_HW_QUEUES=4, HIP's default, so that variable alone cannot
    # say whether a user chose it). Kept at the environment's setting: hipGraph replays
    # (--mode graph, C2's default graph mode) -- the multi-stream captured train step
    # replay faults on the host with 2 queues (profiles/r6l_gpu_tests_segv.log) -- and
    # data-parallel ranks, whose RCCL streams were not measured with fewer queues.
    graphs = args.mode == "graph" or (args.config == "c2" and args.c2_mode == "graph") or \
        (args.config == "c5" and args.c5_mode == "graph")
    if world == 1 and not graphs:
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("OCRK_HW_QUEUES", "2")
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    if args.config in ("c2", "c5"):
        res, elapsed, work = (run_c2 if args.config == "c2" else run_c5)(args, world, rank, device)
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        res["value"] = round(work / elapsed, 2)             # whole job over the slowest rank
        res["ms_per_step"] = round(1e3 * elapsed / (1 if args.config == "c5" else args.steps), 3)
        res["world_size_seen"] = dist.get_world_size() if world > 1 else 1
        if rank == 0:
            print(json.dumps(res), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, _lib
    from cnn_lstm_ctc_ocr_amd.train import Trainer

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    B, W = args.batch, args.width
    T = (W - 2) // 2 - 2
    sizes = RNN_SIZES[args.cell]
    store = ParamStore(ModelConfig(cell=args.cell, rnn_sizes=sizes, dtype=dtype), device=device, seed=0)
    trainer = Trainer(store, sync_bn=args.sync_bn)
    rng = np.random.default_rng(1234 + rank)                # per-rank seed = base + rank
    img, widths, labels = synthetic_batch(rng, B, W, T, device)

    kinds = [args.roofline] + [k for k in args.roofline_also.split(",") if k and k != args.roofline]
    probes = {k: [] for k in kinds}
    table = {}
    op_name, work_fn, op_desc = ROOFLINE_OPS[args.roofline]
    probe = probes[args.roofline]
    op_names = op_name if isinstance(op_name, tuple) else (op_name,)
    # one probe per entry point: kinds sharing an entry point (gemm, dw) cannot both be armed
    armed = {}
    for k in kinds:
        names = ROOFLINE_OPS[k][0]
        for name in (names if isinstance(names, tuple) else (names,)):
            armed.setdefault(name, k)

    def arm_probes():
        for name, k in armed.items():
            fn = ROOFLINE_OPS[k][1]
            _lib.PROBES[name] = (fn[name] if isinstance(fn, dict) else fn, probes[k])
        if args.breakdown:
            for name in _lib.SIGNATURES:
                if name not in op_names and not name.endswith(("_size", "version", "last_error", "tiles")) \
                        and not name.startswith("ocrk_timer"):
                    table[name] = []
                    _lib.PROBES[name] = (None, table[name])

    if args.mode == "graph":
        # one eager step (lazy per-stream state), then the forward + backward is
        # captured with the probe timers inside it as external event nodes
        trainer.step(img, widths, labels)
        arm_probes()
        def drop_warmup_records():          # only the captured launches are timed
            for r in probes.values():
                r.clear()
            for r in table.values():
                r.clear()
        graphed = trainer.graphed(img, widths, labels, before_capture=drop_warmup_records)
        _lib.PROBES.clear()
        run_step = graphed.step
    else:
        run_step = lambda: trainer.step(img, widths, labels)  # noqa: E731
    if args.main_stream == "own":
        # the step on a non-blocking stream of its own instead of the legacy NULL stream:
        # a stream created without hipStreamNonBlocking (a CU-masked one, hipExtStreamCreateWithCUMask)
        # synchronises with the NULL stream, so the step's side work would serialise behind it
        own = torch.cuda.Stream(device)
        own.wait_stream(torch.cuda.current_stream(device))
        step_on_default = run_step

        def run_step():
            with torch.cuda.stream(own):
                return step_on_default()
    for _ in range(args.warmup):
        run_step()
    torch.cuda.synchronize()
    every = 1 if (args.breakdown or args.mode == "graph") else max(1, args.probe_every)
    probed = 0

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if args.mode == "eager":
            # probed steps: the last of every `every` (the last timed step always)
            if (args.steps - 1 - i) % every == 0:
                arm_probes()
                probed += 1
            else:
                _lib.PROBES.clear()
        loss = run_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    _lib.PROBES.clear()
    if args.mode == "graph":
        probed = args.steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    def read(records):
        return [a.elapsed_ms(b) for a, b, _ in records]

    mss = {k: read(r) for k, r in probes.items()}
    if args.mode == "graph":
        # the timers in the graph hold the last timed step; K more replays, each
        # read back after a sync, complete the average over K steps
        rows = {n: read(r) for n, r in table.items() if r}
        for _ in range(args.steps - 1):
            run_step()
            torch.cuda.synchronize()
            for k, r in probes.items():
                mss[k] += read(r)
            for n, r in table.items():
                if r:
                    rows[n] += read(r)
        works = {k: sum(w for _, _, w in r) * args.steps for k, r in probes.items()}
    else:
        rows = {n: read(r) for n, r in table.items() if r}
        works = {k: sum(w for _, _, w in r) for k, r in probes.items()}
    ms, work = mss[args.roofline], works[args.roofline]
    avg_ms = sum(ms) / max(len(ms), 1)
    achieved = work / max(sum(ms), 1e-9) / 1e9          # FLOP/ms -> TFLOP/s
    # bf16 step: the bf16 dense peak; an fp32 store trains with exact f32 MFMA
    # products (train.Trainer -> kernels.f32_exact): the f32 peak
    peak = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS

    if args.breakdown and rank == 0:
        rows = [(n, sum(v) / probed, len(v) // probed) for n, v in rows.items()]
        rows.append(("+".join(op_names), sum(ms) / probed, len(ms) // probed))
        tot = sum(r[1] for r in rows)
        print(f"# per-step device time by entry point (sum {tot:.2f} ms, wall {1e3 * elapsed / args.steps:.2f} ms)",
              file=sys.stderr)
        for n, t, c in sorted(rows, key=lambda r: -r[1]):
            print(f"#  {n:32s} {t:9.3f} ms  {c:4d} calls", file=sys.stderr)

    value = world * B * args.steps / elapsed
    result = {
        "metric": "line-crops/sec (train step) at 32x256 bs=256; CER vs ref",
        "value": round(value, 2),
        "unit": "line-crops/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
        "data": "synthetic (uint8 crops U{0..255}, labels len U{2..19}; random-init weights, reference initialisers)",
        "config": {"workload": "C3: train step (conv+BiLSTM+CTC grad+Adam), LSTM 512/512 (model_bu.py)"
                   if args.cell == "lstm" else
                   "C3 with model.py's cell: train step (conv+BiGRU+CTC grad+Adam), GRU 512/256 (model.py)",
                   "execution": "hipGraph replay of fwd+bwd, eager all-reduce + Adam" if args.mode == "graph"
                   else "eager launches",
                   "global_batch": B * world, "per_gpu_batch": B, "image": f"32x{W}", "seq_len": T,
                   "parallelism": f"dp{world}",
                   "collective": "one bucketed SUM all-reduce of the flat fp32 gradient per step "
                                 "(RCCL over xGMI, backend nccl)" + (" + SyncBN: 8 small all-reduces"
                                                                     if args.sync_bn else "")
                                 if world > 1 else "none",
                   "hip_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "HIP default (4)")},
        "world_size_seen": dist.get_world_size() if world > 1 else 1,
        "roofline": {"bound": "mfma", "kernel": op_desc, "achieved": round(achieved, 2), "peak": round(peak, 1),
                     "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": None,
                     "launches_per_step": len(ms) // max(probed, 1), "avg_launch_ms": round(avg_ms, 4),
                     "algorithmic_flop_per_launch": work / max(len(ms), 1),
                     "timing": "HIP events bracketing each launch on its stream" + (
                         " (external event nodes inside the step graph; last timed step + "
                         f"{args.steps - 1} read-back replays)" if args.mode == "graph" else
                         f" in {probed} of the {args.steps} timed steps (every {every}th)")},
        "loss": round(float(loss.item()), 4),
    }
    if dtype != torch.bfloat16:
        result["roofline"]["peak_note"] = "fp32 training runs exact f32 MFMA products: f32 dense peak"
    for k in kinds[1:]:
        m_k, w_k = mss[k], works[k]
        if not m_k:
            continue
        a_k = w_k / max(sum(m_k), 1e-9) / 1e9
        result.setdefault("roofline_also", []).append(
            {"bound": "mfma", "kernel": ROOFLINE_OPS[k][2], "achieved": round(a_k, 2), "peak": round(peak, 1),
             "unit": "TFLOP/s", "frac": round(a_k / peak, 4), "launches_per_step": len(m_k) // max(probed, 1),
             "avg_launch_ms": round(sum(m_k) / len(m_k), 4), "algorithmic_flop_per_launch": w_k / len(m_k),
             "timing": "HIP events bracketing each launch on its stream (incl. any wait for CUs the "
                       "launch's workgroups spend queued behind other streams' kernels)"})
    if args.roofline == "conv" and os.path.exists(args.traffic_json):
        with open(args.traffic_json) as fh:
            pmc = json.load(fh)
        # the summary counts only while it was taken of the library this run loaded
        lib_sha = hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()
        src = os.path.relpath(args.traffic_json, ROOT)
        if pmc.get("libocrk_sha256") == lib_sha:
            result["roofline"]["traffic"] = pmc["bytes_per_launch"]
            result["roofline"]["traffic_unit"] = "bytes per launch (HBM, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)"
            result["roofline"]["traffic_source"] = f"{src} (PMC passes of this libocrk.so, sha256 {lib_sha[:12]})"
        else:
            result["roofline"]["traffic_note"] = (f"{src} was taken of another libocrk.so build "
                                                  f"({str(pmc.get('libocrk_sha256'))[:12]} vs {lib_sha[:12]}): not reported")
    if rank == 0 and not args.no_cer and args.cell == "lstm":      # the golden decodes are of the LSTM model
        result["cer_vs_ref"] = cer_vs_ref(device)
        if world == 1 and not args.no_trained_cer:
            result["cer_vs_ref_trained"] = cer_vs_ref_trained(device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.cpu_sample, steps=args.cpu_steps, cell=args.cell)
        if args.cell == "lstm":
            result["c1_latency"] = c1_latency(device)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
