"""The C ABI (include/ocrk.h) and its ctypes binding agree, and libocrk.so
loads and exports every declared symbol (no GPU needed: nothing is launched)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ocrk.h")


def _declarations():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    decls = {}
    for m in re.finditer(r"^(int|size_t|uint32_t|const char\*)\s+(ocrk_\w+)\(([^;]*)\);", text, re.M):
        args = m.group(3).strip()
        n = 0 if args in ("", "void") else len(args.split(","))
        decls[m.group(2)] = (m.group(1), n)
    return decls


def test_header_declares_the_abi():
    d = _declarations()
    assert len(d) >= 30
    for name in ("ocrk_ctc_loss", "ocrk_ctc_greedy_decode", "ocrk_conv3x3_fwd", "ocrk_lstm_fwd_step",
                 "ocrk_bn_relu_pool_fwd", "ocrk_gemm", "ocrk_adam"):
        assert name in d


def test_binding_matches_header():
    from cnn_lstm_ctc_ocr_amd import _lib
    d = _declarations()
    assert set(d) == set(_lib.SIGNATURES)
    for name, (_ret, nargs) in d.items():
        assert len(_lib.SIGNATURES[name]) == nargs, name


def test_library_exports_every_symbol():
    from cnn_lstm_ctc_ocr_amd import _lib
    lib = _lib.lib()
    for name in _declarations():
        assert hasattr(lib, name), name
    assert lib.ocrk_version() == 7


def test_no_compute_without_device_pointers():
    """A bad argument is reported through the status + message, not a crash."""
    from cnn_lstm_ctc_ocr_amd import _lib
    with pytest.raises(_lib.InvalidArgumentError, match="T=0"):
        _lib.call("ocrk_ctc_loss", None, None, None, None, 0, 1, 96, 1, 1.0, None, None, None, None, None, 0, None)
    assert _lib.lib().ocrk_ctc_workspace_size(125, 256, 19) == 256 * 2 * 125 * 39 * 4
