"""Dump one trained-weight row's logits and the device beam search's top paths
(wave form and block form) for offline comparison with the literal TF1
restatement (oracle/ref_graph.py ctc_beam_search_single).

    python tools/beam_probe.py OUT.npz BATCH ROW [STEPS]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import trained_model as TM  # noqa: E402
from cnn_lstm_ctc_ocr_amd import decode, model, options  # noqa: E402


def main(out, bi, row, steps=None):
    dev = torch.device("cuda:0")
    batches = TM.shard_batches(TM.TRAIN_SHARD)
    store, _l, _c = TM.train_on_shard(torch.float32, batches, dev, steps=int(steps) if steps else None)
    x, w, _lab = batches[int(bi)]
    with torch.no_grad():
        feats, seq = model.convnet_layers(x.to(dev), w.to(dev), model.INFER, store)
        logits = model.rnn_layers(feats, seq, 95, store).float().contiguous()
    res = {"lg": logits.cpu().numpy(), "seq": seq.cpu().numpy(), "row": int(row)}
    r = int(row)
    one = logits[:, r:r + 1].contiguous()
    s1 = seq[r:r + 1].contiguous()
    for wave in (1, 0):
        for k in (16, 32):
            with options.override(BEAM_WAVE=wave):
                paths, lp = decode.ctc_beam_search_decoder(one, s1, beam_width=k, top_paths=min(k, 16))
            res[f"w{wave}_k{k}_paths"] = np.stack([np.pad(p[0].cpu().numpy(), (0, 200 - p.shape[1]),
                                                          constant_values=-1) for p in paths])
            res[f"w{wave}_k{k}_lp"] = lp.cpu().numpy()[0]
            print(wave, k, lp.cpu().numpy()[0][:4], flush=True)
    np.savez(out, **res)


if __name__ == "__main__":
    main(*sys.argv[1:])
