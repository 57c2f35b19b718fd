"""bench.py's roofline probes (CPU): every probed entry point exists in the C-ABI
table with a work function, and the conv kind counts every conv forward launch of
the bf16 step -- conv1 -> conv2 fused (ocrk_conv12_fwd: both layers' FLOP), the
row-statistics, ReLU-bit and plain conv entries -- at SURVEY 8(d)'s per-pixel FLOP."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from cnn_lstm_ctc_ocr_amd import _lib  # noqa: E402


def test_probed_entries_are_abi_entries_with_work():
    for kind, (names, fn, desc) in bench.ROOFLINE_OPS.items():
        names = names if isinstance(names, tuple) else (names,)
        for n in names:
            assert n in _lib.SIGNATURES, (kind, n)
            f = fn[n] if isinstance(fn, dict) else fn
            assert callable(f), (kind, n)
        assert desc


def test_conv_kind_flop_per_launch():
    names, fn, _ = bench.ROOFLINE_OPS["conv"]
    assert set(names) >= {"ocrk_conv12_fwd", "ocrk_conv3x3_fwd", "ocrk_conv3x3_fwd_rowstats",
                          "ocrk_conv3x3_fwd_relu_bits"}
    B, IH, IW = 256, 32, 256
    # ocrk_conv12_fwd(x, x_is_u8, B, IH, IW, ...): conv1 (1 -> 32) + conv2 (32 -> 32), valid conv1
    got = fn["ocrk_conv12_fwd"]((None, 1, B, IH, IW) + (None,) * 10)
    assert got == 2.0 * B * 30 * 254 * 9 * (32 + 32 * 32)
    assert len(_lib.SIGNATURES["ocrk_conv12_fwd"]) == 15
    # (x, B, H, W, cin, w_nk, bias, cout, ...): conv6 at C3
    for n in ("ocrk_conv3x3_fwd", "ocrk_conv3x3_fwd_rowstats", "ocrk_conv3x3_fwd_relu_bits"):
        args = (None, B, 7, 126, 128, None, None, 128) + (None,) * (len(_lib.SIGNATURES[n]) - 8)
        assert fn[n](args) == 2.0 * B * 7 * 126 * 9 * 128 * 128
