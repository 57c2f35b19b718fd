"""Launch-shape logic of the weight-gradient GEMMs (host only, no GPU):
model._splits' K slices keep every 256 x 256 TN launch within its item cap
(one round on the chip by default) and the slices cover K; the per-layer caps
(options TN_ITEMS_L1 / TN_ITEMS_LATE, model._tn_items) feed it."""
import pytest

from cnn_lstm_ctc_ocr_amd import model, options


def _items(M, N, splits, batch):
    return -(-M // 256) * -(-N // 256) * batch * splits


@pytest.mark.parametrize("M,N,batch", [(256, 2048, 2), (512, 2048, 2), (1024, 2048, 2), (512, 1024, 2),
                                       (1024, 1024, 2), (256, 1024, 1)])
@pytest.mark.parametrize("cap", [None, 256, 192, 128])
def test_splits_stay_within_the_item_cap(M, N, batch, cap):
    R = 32000
    s = model._splits(M, N, R, batch=batch, items=cap)
    assert s >= 1
    assert _items(M, N, s, batch) <= max(cap or options.get("TN_ITEMS"), -(-M // 256) * -(-N // 256) * batch)
    assert R // s >= 1024 or s == 1                 # slices of >= 1024 rows
    # the host wrapper rounds the slice to 32 rows; the slices still cover K
    kc = -(-(-(-R // s)) // 32) * 32
    assert kc * -(-R // kc) >= R


def test_default_caps_fill_one_round_at_the_bench_shapes():
    R = 32000
    for M in (256, 512, 1024):
        s = model._splits(M, 2048, R, batch=2)
        assert _items(M, 2048, s, 2) == 256


def test_per_layer_caps(ocrk_opts):
    from cnn_lstm_ctc_ocr_amd import options
    ocrk_opts("TN_ITEMS_L1", 128)
    assert model._tn_items(1) == 128
    assert model._tn_items(2) == options.get("TN_ITEMS")
    s = model._splits(256, 2048, 32000, batch=2, items=model._tn_items(1))
    assert _items(256, 2048, s, 2) == 128
