"""ctypes binding of libocrk_comm.so (include/ocrk_comm.h): the optional RCCL
all-reduce of the data-parallel gradient exchange as a C ABI.

The trainer's own exchange stays torch.distributed (backend "nccl" = RCCL,
train.GradBuckets); this is the same collective for a host that binds the C ABI
(INTEGRATION.md shows the TF-side form). One Communicator per process and GPU:

    uid = unique_id()                      # rank 0; broadcast the bytes to every rank
    comm = Communicator(world, rank, uid, device_index)
    comm.allreduce_(flat_grad)             # in place, on torch's current stream
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OCRK_COMM_LIB") or os.path.join(_HERE, "libocrk_comm.so")
ID_BYTES = 128
_DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float64: 2, torch.int32: 3}

_p, _i32, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
SIGNATURES = {
    "ocrk_comm_version": [],
    "ocrk_comm_unique_id": [_p],
    "ocrk_comm_init": [ctypes.POINTER(ctypes.c_void_p), _i32, _i32, _p, _i32],
    "ocrk_comm_info": [_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
    "ocrk_allreduce_sum": [_p, _sz, _i32, _p, _p],
    "ocrk_comm_destroy": [_p],
    "ocrk_comm_last_error": [],
}
_lib = None


class CommError(RuntimeError):
    pass


def lib():
    """The loaded libocrk_comm.so (built by `make`; no fallback: a missing library raises)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CommError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build())")
        h = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            f = getattr(h, name)
            f.argtypes = args
            f.restype = ctypes.c_char_p if name == "ocrk_comm_last_error" else ctypes.c_int
        _lib = h
    return _lib


def _check(status):
    if status != 0:
        raise CommError(f"ocrk_comm status {status}: {lib().ocrk_comm_last_error().decode(errors='replace')}")


def unique_id():
    """Rank 0's rendezvous token (ncclGetUniqueId): ID_BYTES bytes for every rank."""
    buf = ctypes.create_string_buffer(ID_BYTES)
    _check(lib().ocrk_comm_unique_id(buf))
    return buf.raw


class Communicator:
    """This process's RCCL communicator on one GPU (ocrk_comm_init)."""

    def __init__(self, world, rank, uid, device=0):
        if len(uid) != ID_BYTES:
            raise ValueError(f"unique id must be {ID_BYTES} bytes, got {len(uid)}")
        self.device = torch.device("cuda", device)
        h = ctypes.c_void_p()
        _check(lib().ocrk_comm_init(ctypes.byref(h), int(world), int(rank), ctypes.c_char_p(bytes(uid)), int(device)))
        self._h = h

    def info(self):
        w, r = ctypes.c_int(), ctypes.c_int()
        _check(lib().ocrk_comm_info(self._h, ctypes.byref(w), ctypes.byref(r)))
        return w.value, r.value

    def allreduce_(self, t):
        """t = the sum of t over the ranks, in place, on torch's current stream."""
        if not (t.is_cuda and t.is_contiguous()) or t.dtype not in _DTYPES:
            raise ValueError("allreduce_ needs a contiguous cuda tensor of float32 / bfloat16 / float64 / int32")
        stream = torch.cuda.current_stream(t.device).cuda_stream
        _check(lib().ocrk_allreduce_sum(ctypes.c_void_p(t.data_ptr()), t.numel(), _DTYPES[t.dtype], self._h,
                                        ctypes.c_void_p(stream)))
        return t

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _check(lib().ocrk_comm_destroy(self._h))
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
