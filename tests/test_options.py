"""The engine-option registry (include/ocrk.h ocrk_get_option / ocrk_set_option,
cnn_lstm_ctc_ocr_amd/options.py): every kernel-side name the Python layer
forwards is known to libocrk and listed in the header, set / override restore
the previous value, and unknown names fail loudly. No GPU: the registry is
host state of the library."""
import os
import re

import pytest

from cnn_lstm_ctc_ocr_amd import options

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "ocrk.h")


def test_every_kernel_option_is_registered_and_documented():
    text = open(HEADER).read()
    listed = re.search(r"Names: (.*?)\(meanings in", text, re.S).group(1)
    names = {n.strip(" *\n,") for n in re.split(r"[,\s]+", listed) if n.strip(" *\n,")}
    assert set(options.KERNEL_OPTIONS) == names
    for name in options.KERNEL_OPTIONS:
        v = options.get(name)
        assert isinstance(v, int)


def test_set_and_override_restore():
    before = options.get("BN_BWD_BLOCKS")
    with options.override(BN_BWD_BLOCKS=512, CONV_SIDE=0):
        assert options.get("BN_BWD_BLOCKS") == 512
        assert options.get("CONV_SIDE") == 0
    assert options.get("BN_BWD_BLOCKS") == before
    assert options.get("CONV_SIDE") == 1
    prev = options.set("GEMM_TN", 0)
    try:
        assert options.get("GEMM_TN") == 0
    finally:
        options.set("GEMM_TN", prev)


def test_unknown_option_raises():
    with pytest.raises(KeyError):
        options.get("NO_SUCH_OPTION")
    with pytest.raises(KeyError):
        options.set("NO_SUCH_OPTION", 1)
