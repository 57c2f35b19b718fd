"""Training-regime sweep for the trained-weight tests (VERDICT r5 "next" #1: the
fp32 shard CER was non-monotone, 0.18 -> 0.33 over steps 2,000-2,500).

Trains the seed-0 LSTM 512/512 on the data/val shard under several schedules and
two library variants (the pooled-output BN backward and the z walk, whose
gradients differ only in summation order) and records, every 500 steps, the
shard CER in INFER mode (BN moving averages, what the tests and the server use)
and in TRAIN mode (batch statistics), plus the held-out data/test CER at the end.

    python tools/trained_sweep.py OUT.json [variant ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import trained_model as TM  # noqa: E402
from cnn_lstm_ctc_ocr_amd import model, options  # noqa: E402

VARIANTS = {
    # name: (dtype, regime overrides, options)
    "r5": ("f32", dict(steps=2500), {}),
    "r5_z": ("f32", dict(steps=2500), dict(POOLED_BN=0, BN_ROUTE_NCH=8)),
    "a": ("f32", dict(steps=4000), {}),
    "a_z": ("f32", dict(steps=4000), dict(POOLED_BN=0, BN_ROUTE_NCH=8)),
    "a_order8": ("f32", dict(steps=4000, order_seed=8), {}),
    "b": ("f32", dict(steps=4000, decay_steps=700), {}),
    "b_z": ("f32", dict(steps=4000, decay_steps=700), dict(POOLED_BN=0, BN_ROUTE_NCH=8)),
    "a_bf16": ("bf16", dict(steps=4000), {}),
}


def main(out, names):
    dev = torch.device("cuda:0")
    train = TM.shard_batches(TM.TRAIN_SHARD)
    held = TM.shard_batches(TM.HELD_OUT_SHARD, drop_remainder=False)
    res = {}
    for name in names or list(VARIANTS):
        dt, over, opts = VARIANTS[name]
        dtype = torch.float32 if dt == "f32" else torch.bfloat16
        tr_dev = TM.to_device(train, dev, dtype)
        held_dev = TM.to_device(held, dev, dtype)
        t0 = time.time()
        with options.override(**opts):
            store, losses, curves = TM.train_on_shard(
                dtype, train, dev, evals={"infer": lambda s: TM.shard_cer(s, tr_dev),
                                          "train_mode": lambda s: TM.shard_cer(s, tr_dev, model.TRAIN)}, **over)
            held_cer = TM.shard_cer(store, held_dev)
        w = losses.reshape(-1, 50).mean(1)
        res[name] = dict(dtype=dt, regime={**TM.REGIME, **over}, options=opts, infer_cer=curves["infer"],
                         train_mode_cer=curves["train_mode"], held_out_cer=held_cer,
                         window_mean=[round(float(v), 3) for v in w], seconds=round(time.time() - t0, 1))
        print(f"{name}: infer {[(s, round(c, 3)) for s, c in curves['infer']]}\n"
              f"   train-mode {[(s, round(c, 3)) for s, c in curves['train_mode']]}\n"
              f"   held-out {held_cer:.3f}  windows {[round(float(v), 2) for v in w[::10]]}  "
              f"{time.time() - t0:.0f}s", flush=True)
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)
        del store
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
