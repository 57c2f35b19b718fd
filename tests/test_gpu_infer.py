"""infer.InferGraph: the graph-captured INFER forward (+ CTC loss + greedy
decode) replays exactly the eager launches -- same logits, loss and decodes --
for a new batch copied into its static buffers, at the C2 shape (fp32, B=64,
32x256) and a ragged-width bf16 bucket; and it refuses to replay once the
variables have changed."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _eager(store, img, widths, labels):
    from cnn_lstm_ctc_ocr_amd import decode, model
    with torch.no_grad():
        feats, seq = model.convnet_layers(img, widths, model.INFER, store)
        logits = model.rnn_layers(feats, seq, 95, store)
        loss = model.ctc_loss_layer(logits, labels, seq, check=False) if labels is not None else None
        dec, dlen, _ = decode.ctc_greedy_decoder_raw(logits, seq)
    return logits, seq, loss, dec, dlen


@pytest.mark.parametrize("dtype,B,W,ragged", [(torch.float32, 64, 256, False), (torch.bfloat16, 32, 160, True)])
def test_infer_graph_replays_the_eager_forward(cuda, dtype, B, W, ragged):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore, kernels as K
    from cnn_lstm_ctc_ocr_amd.infer import InferGraph
    store = ParamStore(ModelConfig(dtype=dtype), device=cuda, seed=3)
    rng = np.random.default_rng(77)

    def batch():
        img = torch.from_numpy(rng.integers(0, 256, (B, 32, W, 1), dtype=np.uint8)).to(cuda)
        w = rng.integers(W - 31, W + 1, B) if ragged else np.full(B, W)
        w = torch.from_numpy(w.astype(np.int32)).to(cuda)
        lab = torch.from_numpy(rng.integers(0, 95, (B, 6)).astype(np.int32)).to(cuda)
        ln = torch.from_numpy(rng.integers(2, 7, B).astype(np.int32)).to(cuda)
        return img, w, (lab, ln)
    img0, w0, lab0 = batch()
    g = InferGraph(store, image=img0.clone(), widths=w0.clone(), labels=(lab0[0].clone(), lab0[1].clone()),
                   n_classes=95)
    K.status_word(cuda).zero_()
    for _ in range(2):                                   # a fresh batch each replay
        img, w, (lab, ln) = batch()
        g.labels[0].copy_(lab)
        g.labels[1].copy_(ln)
        g.run(img, w)
        logits, seq, loss, dec, dlen = _eager(store, img, w, (lab, ln))
        torch.cuda.synchronize()
        assert torch.equal(g.logits, logits)
        assert torch.equal(g.seq_len.to(torch.int32), seq.to(torch.int32)) and torch.isfinite(g.loss)
        assert torch.allclose(g.loss, loss, rtol=1e-6, atol=0)
        assert torch.equal(g.decoded, dec) and torch.equal(g.decoded_len, dlen)
    assert K.read_status(cuda) == 0
    with pytest.raises(ValueError):
        g.run(img[:, :, :W // 2].contiguous())
    store.bump()
    with pytest.raises(RuntimeError):
        g.replay()
