"""Weight images of a parameter version (ParamStore.images): the one batched
ocrk_copy_batch launch (LDS job search; float4 reads and packed writes on the
aligned jobs, the scalar form on the 95-column logits) writes exactly the
bits of the per-image builders (ocrk_permute3 / ocrk_strided_copy), for both
cells and both storage types, and again after an update (bump)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _all_images(store, dtype):
    out = []
    for li in range(2, 9):
        out += list(store.conv_images(f"conv{li}", dtype))
    for layer in range(1, len(store.cfg.rnn_sizes) + 1):
        imgs = store.lstm_images(layer, dtype) if store.cfg.cell == "lstm" else store.gru_images(layer, dtype)
        out += [t for t in imgs if t.dtype == dtype]
    out += [store.logits_image(dtype), store.logits_image_t(dtype)]
    return [t.clone() for t in out]


@pytest.mark.parametrize("cell,sizes", [("lstm", (512, 512)), ("gru", (512, 256))])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_batched_images_equal_the_per_image_builders(cuda, cell, sizes, dtype):
    from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore
    store = ParamStore(ModelConfig(cell=cell, rnn_sizes=sizes, dtype=dtype), device=cuda, seed=7)
    for rnd in range(2):
        batched = _all_images(store, dtype)
        assert store._plan_fresh                          # the batched launch made them
        plan, store._plan = store._plan, None             # the per-image builders (the path of keys
        store._plan_for = lambda key: None                # outside the batched plan)
        store._images.clear()
        built = _all_images(store, dtype)
        del store._plan_for
        store._plan = plan
        torch.cuda.synchronize()
        assert len(batched) == len(built)
        for a, b in zip(batched, built):
            assert a.shape == b.shape and torch.equal(a, b)
        with torch.no_grad():                             # an update: new values, new images
            store.flat.mul_(1.5).add_(0.01)
        store.bump()
