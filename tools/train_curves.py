"""Training-curve sweeps beside tests/test_gpu_trained.py (any step count / lr):
the same fixture (the reference's data/val/words-000.tfrecord crops), the same
width-sorted batches of 32 and seeded epoch shuffle, both precisions from the
same seed, `--steps` steps at `--lr`, the loss of every step and the greedy CER
on the shard every `--eval-every` steps, written as JSON.

    python tools/train_curves.py --steps 2000 --lr 1e-3 --out gpurun_out/curves.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--eval-every", type=int, default=250)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, decode, model
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    from test_gpu_trained import shard_batches
    dev = torch.device("cuda:0")
    batches = shard_batches()
    res = {"steps": args.steps, "lr": args.lr, "batches": len(batches), "batch": 32,
           "data": "tests/golden/mjsynth_val_words000.npz (reference data/val/words-000.tfrecord, 803 crops)"}
    for name, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=dt), device=dev, seed=0)
        tr = Trainer(store, learning_rate=args.lr)
        rng = np.random.default_rng(7)
        dbs = [(img.to(device=dev, dtype=dt), w, lab) for img, w, lab in batches]
        order = []
        while len(order) < args.steps:
            order += list(rng.permutation(len(dbs)))
        losses, cers = [], []

        def cer():
            edits, total = 0.0, 0
            with torch.no_grad():
                for img, w, lab in dbs:
                    feats, seq = model.convnet_layers(img, w, model.INFER, store)
                    logits = model.rnn_layers(feats, seq, 95, store).float()
                    hyp = decode.ctc_greedy_decoder(logits, seq)[0][0]
                    ref, ref_len = model.dense_labels(lab, len(lab), dev)
                    d = decode.edit_distance(hyp, (hyp >= 0).sum(1).to(torch.int32), ref, ref_len)
                    edits += float(d.sum())
                    total += int(ref_len.sum())
            return edits / total
        t0 = time.time()
        for s, i in enumerate(order[:args.steps], start=1):
            img, w, lab = dbs[i]
            losses.append(tr.step(img, w, lab))
            if s % args.eval_every == 0:
                cers.append((s, cer()))
                print(f"# {name} step {s}: loss {float(losses[-1]):.3f} CER {cers[-1][1]:.4f} "
                      f"({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
        tr.check_status()
        res[name] = {"loss": [round(float(v), 4) for v in torch.stack(losses).cpu()], "cer": cers}
    l32, l16 = np.array(res["fp32"]["loss"]), np.array(res["bf16"]["loss"])
    w = 50
    m32, m16 = l32[:len(l32) // w * w].reshape(-1, w).mean(1), l16[:len(l16) // w * w].reshape(-1, w).mean(1)
    res["window"] = w
    res["window_rel_diff"] = [round(float(v), 5) for v in np.abs(m16 - m32) / m32]
    with open(args.out, "w") as fh:
        json.dump(res, fh)
    print(json.dumps({"max_window_rel_diff": max(res["window_rel_diff"]), "cer_fp32": res["fp32"]["cer"][-1],
                      "cer_bf16": res["bf16"]["cer"][-1]}))


if __name__ == "__main__":
    main()
