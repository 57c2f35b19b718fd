"""The optional RCCL all-reduce C ABI (include/ocrk_comm.h, libocrk_comm.so): the
header, the ctypes table and the library agree, and argument errors come back as
status + message (CPU: nothing is launched, no communicator is created)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ocrk_comm.h")


def _declarations():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"^(int|const char\*)\s+(ocrk_\w+)\(([^;]*)\);", text, re.M):
        args = m.group(3).strip()
        out[m.group(2)] = 0 if args in ("", "void") else len(args.split(","))
    return out


def test_header_binding_library_agree():
    from cnn_lstm_ctc_ocr_amd import comm
    d = _declarations()
    assert set(d) == set(comm.SIGNATURES)
    for name, n in d.items():
        assert len(comm.SIGNATURES[name]) == n, name
    lib = comm.lib()
    for name in d:
        assert hasattr(lib, name), name
    assert lib.ocrk_comm_version() == 1


def test_argument_errors_are_reported():
    from cnn_lstm_ctc_ocr_amd import comm
    lib = comm.lib()
    h = ctypes.c_void_p()
    uid = ctypes.create_string_buffer(comm.ID_BYTES)
    assert lib.ocrk_comm_init(ctypes.byref(h), 2, 5, uid, 0) == 1
    assert b"rank 5 outside world 2" in lib.ocrk_comm_last_error()
    assert lib.ocrk_allreduce_sum(None, 4, 0, None, None) == 1
    assert b"null communicator" in lib.ocrk_comm_last_error()
    assert lib.ocrk_comm_unique_id(None) == 1
    assert lib.ocrk_comm_destroy(None) == 0
    with pytest.raises(ValueError):
        comm.Communicator(1, 0, b"short")
