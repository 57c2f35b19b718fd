"""Training past the blank plateau, and parity at TRAINED weights.

The reference trains (src/weinman/train.py:168-201) and serves a trained model
(src/processing/server.py:98-99); at the reference initialisers the ReLU logits
are nearly degenerate, so decode parity there is checked only on easy rows.
Here the LSTM 512/512 model is trained from seed 0 on the reference's own data
-- every crop of data/val/words-000.tfrecord (tests/golden/
mjsynth_val_words000.npz, tools/make_val_fixture.py) through the training input
semantics (first-row pad, 0.0 dynamic padding, mjsynth.py:185-194) in
width-sorted batches of 32, a seeded shuffle per epoch -- for STEPS
Trainer.step calls (Adam with the reference's exponential decay,
train.py:120-137, at LR = 1e-3 instead of the reference's 1e-4 so the run
leaves the blank plateau in ~1,500 steps instead of tens of thousands, and
the decay scaled to the short run -- rate 0.5 per 1,000 steps instead of 0.9
per 2^16 -- so the last evaluations are not taken on a 10x rate's noise), in
fp32 (the reference's precision) and in bf16 (the benched precision). Then:

* the fp32 model's shard CER (greedy, validate.py:81-92; CER = total edit
  distance / total label length, test.py:90-99) must be far below the
  plateau's 1.0;
* its weights are copied to the host and the reference graph is run in
  float64 (oracle/torch_ref.py, pinned to the NumPy oracle in
  tests/test_oracle.py) on the golden test bucket (serving uint8 and training
  float forms) and on every crop of the shard in its 25 width-sorted batches (800 crops,
  widths 37-330):
  logits <= 1e-4 relative L2, greedy and beam-16 decodes compared on EVERY row:
  a row may differ only where the float64 graph has a near-tie (a frame's top-2
  logits within 1e-4 of the largest logit, or a top-2 beam gap <= 1e-3), and
  such rows stay <= 2 % (measured on MI355X: 0 of 816 differ; 8 rows carry a greedy
  near-tie and still agree);
* bf16 and fp32 runs agree step for step before the plateau (50-step window
  means within 5 % over the first 1,000 steps) and both end well below CER 1
  with CERs within 0.10 of each other (the trajectories separate once the
  models leave the plateau: a different rounding of one update changes which
  crops are learned first).

$OCRK_CURVES_OUT, when set, receives the curves, CERs and parity counts as JSON.
"""
import json
import multiprocessing as mp
import os

import numpy as np
import pytest
import torch

from oracle import ref_graph as G

pytestmark = pytest.mark.gpu
STEPS = 2500
LR = 1e-3
DECAY_RATE, DECAY_STEPS = 0.5, 1000
WINDOW = 50
EARLY = 1000              # steps before either run leaves the blank plateau
EVAL_EVERY = 500
VAL_BATCHES = tuple(range(25))  # every crop of the shard: 25 width-sorted batches of 32 (widths 37-330)
FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "mjsynth_val_words000.npz")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "mjsynth_test_bucket.npz")
_REPORT = {}


def shard_batches():
    """The shard as 25 width-sorted host batches (image f32 [32, H, W, 1], widths i32 [32], labels)."""
    from cnn_lstm_ctc_ocr_amd import input_pipeline as P
    g = np.load(FIXTURE)
    order = np.argsort(g["widths"], kind="stable")
    items = []
    for i in order:
        o, w, h = int(g["offsets"][i]), int(g["widths"][i]), int(g["heights"][i])
        crop = g["pixels"][:h, o:o + w, None]
        n = int(g["label_len"][i])
        items.append({"image": P.preprocess_image(crop), "width": w, "labels": g["labels"][i, :n].tolist(),
                      "length": n, "text": str(g["texts"][i]), "filename": str(i)})
    out = []
    for k in range(len(items) // 32):
        image, width, _label, _len, _text, _fn = P.make_batch(items[32 * k:32 * k + 32])
        out.append((image, width, [it["labels"] for it in items[32 * k:32 * k + 32]]))
    return out


def shard_cer(store, dev_batches):
    from cnn_lstm_ctc_ocr_amd import decode, model
    edits, total = 0.0, 0
    with torch.no_grad():
        for img, w, lab in dev_batches:
            feats, seq = model.convnet_layers(img, w, model.INFER, store)
            logits = model.rnn_layers(feats, seq, 95, store).float()
            hyp = decode.ctc_greedy_decoder(logits, seq)[0][0]
            ref, ref_len = model.dense_labels(lab, len(lab), img.device)
            d = decode.edit_distance(hyp, (hyp >= 0).sum(1).to(torch.int32), ref, ref_len)
            edits += float(d.sum())
            total += int(ref_len.sum())
    return edits / total


def train_on_shard(dtype, batches, device, steps=STEPS, lr=LR, eval_every=EVAL_EVERY):
    """Seed-0 LSTM 512/512 trained `steps` Trainer.steps on the shard; returns
    (store, per-step losses, [(step, shard CER)])."""
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    from cnn_lstm_ctc_ocr_amd.train import Trainer
    store = ParamStore(ModelConfig(cell="lstm", rnn_sizes=(512, 512), dtype=dtype), device=device, seed=0)
    tr = Trainer(store, learning_rate=lr, decay_rate=DECAY_RATE, decay_steps=DECAY_STEPS)
    rng = np.random.default_rng(7)
    dev = [(img.to(device=device, dtype=dtype), w, lab) for img, w, lab in batches]
    order = []
    while len(order) < steps:
        order += list(rng.permutation(len(dev)))
    losses, cers = [], []
    for s, i in enumerate(order[:steps], start=1):
        img, w, lab = dev[i]
        losses.append(tr.step(img, w, lab).detach())
        if s % eval_every == 0 or s == steps:
            cers.append((s, shard_cer(store, dev)))
    tr.check_status()
    return store, np.array([float(v) for v in torch.stack(losses).cpu()]), cers


@pytest.fixture(scope="module")
def shard():
    return shard_batches()


@pytest.fixture(scope="module")
def fp32_run(cuda, shard):
    return train_on_shard(torch.float32, shard, cuda)


@pytest.fixture(scope="module")
def bf16_run(cuda, shard):
    return train_on_shard(torch.bfloat16, shard, cuda)


def _write_report():
    path = os.environ.get("OCRK_CURVES_OUT")
    if path:
        with open(path, "w") as fh:
            json.dump(_REPORT, fh)


def test_fp32_leaves_blank_plateau(fp32_run):
    _store, losses, cers = fp32_run
    w = losses.reshape(-1, WINDOW).mean(1)
    _REPORT.update(steps=STEPS, lr=LR, decay=(DECAY_RATE, DECAY_STEPS), window=WINDOW, fp32_loss=[round(v, 4) for v in losses.tolist()],
                   fp32_window_mean=w.tolist(), fp32_cer=[(int(a), float(b)) for a, b in cers])
    _write_report()
    print(f"fp32 windows {np.round(w[::5], 2).tolist()}\nfp32 CER {cers}")
    assert np.isfinite(losses).all()
    # the plateau decodes nothing (CER 1.0). The 2,500-step trajectory at 10x the reference's
    # rate is sensitive to summation order: the same seed and data end at CER 0.144 with the
    # z-walk BN backward (OCRK_POOLED_BN=0 OCRK_BN_ROUTE_NCH=8) and 0.202 with the default
    # pooled-output pass (gradients within 1e-5 of each other, test_bn_bwd_pooled_matches_z_form)
    assert cers[-1][1] < 0.3, cers
    assert w[-1] < 0.2 * w[EARLY // WINDOW - 1]


def _beam_rows(args):
    lg, sl = args
    paths, lp = G.ctc_beam_search_decode(lg, sl, beam_width=16, top_paths=2)
    return paths[0][0], lp[0]


def _near_tie_frames(lg, n, tol):
    """frames t < n whose top-2 logits differ by <= tol (exact 0 = 0 ReLU ties included)"""
    top2 = np.sort(lg[:n], axis=1)[:, -2:]
    return int(np.sum(top2[:, 1] - top2[:, 0] <= tol))


def test_trained_fp32_parity_vs_float64_graph(cuda, fp32_run, shard):
    from cnn_lstm_ctc_ocr_amd import decode, model
    from oracle.torch_ref import TorchRef
    store = fp32_run[0]
    ref = TorchRef({k: v.astype(np.float64) for k, v in store.state_dict().items()}, (512, 512), torch.float64)
    g = np.load(GOLDEN)
    cases = [("test_u8", torch.from_numpy(g["x_u8"]), g["widths"]),
             ("test_f32", torch.from_numpy(g["x_f32"]), g["widths"])]
    cases += [(f"val{i}", shard[i][0], shard[i][1].numpy()) for i in VAL_BATCHES]
    rows = []
    for name, x, w in cases:
        with torch.no_grad():
            feats, seq = model.convnet_layers(x.to(cuda), torch.as_tensor(w).to(cuda), model.INFER, store)
            logits = model.rnn_layers(feats, seq, 95, store)
            greedy = decode.ctc_greedy_decoder(logits, seq)[0][0].cpu().numpy()
            beam, logp = decode.ctc_beam_search_decoder(logits, seq, beam_width=16)
            lr = ref.forward(x, training=False, widths=w).numpy()
        seq = seq.cpu().numpy()
        assert seq.tolist() == ref.seq_len.tolist(), name
        lg = logits.cpu().numpy()
        err = np.linalg.norm(lg - lr) / np.linalg.norm(lr)
        assert err < 1e-4, (name, err)
        for b in range(lg.shape[1]):
            e = np.linalg.norm(lg[:, b] - lr[:, b]) / np.linalg.norm(lr[:, b])
            assert e < 3e-4, (name, b, e)
        got_b = beam[0].cpu().numpy()
        greedy_ref, _ = G.ctc_greedy_decode(lr, seq)
        greedy_dev, _ = G.ctc_greedy_decode(lg, seq)
        tol = 1e-4 * max(1.0, float(np.abs(lr).max()))
        for b in range(lg.shape[1]):
            rows.append(dict(case=name, row=b, seq=int(seq[b]), lg=lg[:, b:b + 1], lr=lr[:, b:b + 1],
                             greedy=greedy[b][greedy[b] >= 0].tolist(), greedy_dev=greedy_dev[b],
                             greedy_ref=greedy_ref[b], beam=got_b[b][got_b[b] >= 0].tolist(),
                             logp=float(logp[b, 0]), ties=_near_tie_frames(lr[:, b], int(seq[b]), tol)))
    jobs = []
    for r in rows:
        sl = np.array([r["seq"]])
        jobs += [(r["lg"], sl), (r["lr"], sl)]
    with mp.get_context("spawn").Pool(min(16, len(jobs))) as pool:
        res = pool.map(_beam_rows, jobs, chunksize=2)
    n = len(rows)
    greedy_ties = greedy_diff = beam_ties = beam_diff = 0
    for k, r in enumerate(rows):
        (p_dev, lp_dev), (p_ref, lp_ref) = res[2 * k], res[2 * k + 1]
        where = (r["case"], r["row"])
        # the decoders bit-exact on the device's own logits
        assert r["greedy"] == r["greedy_dev"], where
        assert r["beam"] == p_dev, where
        np.testing.assert_allclose(r["logp"], lp_dev[0], rtol=1e-4, atol=2e-3, err_msg=str(where))
        # end to end against the float64 graph, near-ties counted
        if r["greedy"] != r["greedy_ref"]:
            greedy_diff += 1
            assert r["ties"] > 0, (where, r["greedy"], r["greedy_ref"])
        greedy_ties += r["ties"] > 0
        if r["beam"] != p_ref:
            beam_diff += 1
            assert lp_ref[0] - lp_ref[1] <= 1e-3, (where, r["beam"], p_ref, lp_ref)
        beam_ties += lp_ref[0] - lp_ref[1] <= 1e-3
    greedy_ties, beam_ties = int(greedy_ties), int(beam_ties)
    print(f"trained-weight parity: {n} rows; greedy near-tie rows {greedy_ties}, differing {greedy_diff}; "
          f"beam-16 near-tie rows {beam_ties}, differing {beam_diff}")
    _REPORT.update(parity_rows=n, greedy_near_tie_rows=greedy_ties, greedy_differs=greedy_diff,
                   beam_near_tie_rows=beam_ties, beam_differs=beam_diff,
                   parity_cases={name: int(len(w)) for name, _x, w in cases})
    _write_report()
    # every row is compared; a row may differ only where the float64 graph itself has a
    # near-tie (asserted above), and such excluded rows stay <= 2 % (measured: 0 of 816)
    assert greedy_diff <= 0.02 * n and beam_diff <= 0.02 * n, (greedy_diff, beam_diff, n)


def test_bf16_trains_like_fp32_on_reference_shard(fp32_run, bf16_run):
    _s32, l32, c32 = fp32_run
    _s16, l16, c16 = bf16_run
    w32 = l32.reshape(-1, WINDOW).mean(1)
    w16 = l16.reshape(-1, WINDOW).mean(1)
    rel = np.abs(w16 - w32) / w32
    early = rel[:EARLY // WINDOW]
    _REPORT.update(bf16_loss=[round(v, 4) for v in l16.tolist()], bf16_window_mean=w16.tolist(),
                   window_rel_diff=rel.tolist(), bf16_cer=[(int(a), float(b)) for a, b in c16])
    _write_report()
    print(f"early windows max rel {early.max():.4f}; CER fp32 {c32[-1][1]:.4f} bf16 {c16[-1][1]:.4f}")
    assert np.isfinite(l16).all()
    assert early.max() < 0.05, early
    assert c32[-1][1] < 0.25 and c16[-1][1] < 0.25, (c32, c16)
    assert abs(c16[-1][1] - c32[-1][1]) < 0.10, (c32, c16)
