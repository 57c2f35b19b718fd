"""ctypes binding of libocrk.so (the C ABI declared in include/ocrk.h).

The library is built in-tree by ``make`` (or ``__graft_entry__.build()``).
There is no fallback: if the shared object is missing or stale this module
raises, so a GPU run can never silently route through a CPU path.

``torch`` is imported first on purpose: libocrk.so links libamdhip64.so.7 and
must bind to the same HIP runtime instance torch already loaded (identical
SONAME), so device pointers and streams are shared between the two.
"""
import ctypes
import os

import torch  # noqa: F401  (see module docstring: runtime must be torch's)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OCRK_LIB") or os.path.join(_HERE, "libocrk.so")   # OCRK_LIB: experiment builds

OCRK_OK = 0
OCRK_ERR_INVALID_ARG = 1
OCRK_ERR_HIP = 2
OCRK_ERR_INFEASIBLE = 3

F32 = 0
BF16 = 1

_p = ctypes.c_void_p
_i32 = ctypes.c_int
_u32 = ctypes.c_uint
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_sz = ctypes.c_size_t

# name -> argtypes (restype is int unless listed in _RESTYPE).
SIGNATURES = {
    "ocrk_version": [],
    "ocrk_last_error": [],
    "ocrk_set_option": [ctypes.c_char_p, _i64, _p],
    "ocrk_get_option": [ctypes.c_char_p, _p],
    "ocrk_preprocess": [_p, _i64, _p, _i32, _p],
    "ocrk_status_clear": [_p, ctypes.c_uint32, _p],
    "ocrk_set_f32_gemm_mode": [_i32],
    "ocrk_f32_gemm_exact": [],
    "ocrk_ctc_workspace_size": [_i32, _i32, _i32],
    "ocrk_ctc_loss": [_p, _p, _p, _p, _i32, _i32, _i32, _i32, _f32, _p, _p, _p, _p, _p, _sz, _p],
    "ocrk_ctc_greedy_decode": [_p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p],
    "ocrk_ctc_beam_workspace_size": [_i32, _i32, _i32],
    "ocrk_gru_fwd_step": [_p, _p, _p, _p, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p],
    "ocrk_gru_fwd": [_p, _p, _p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p],
    "ocrk_gru_bwd": [_p, _p, _p, _p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p],
    "ocrk_ctc_beam_decode": [_p, _p, _i32, _i32, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _sz, _p],
    "ocrk_crc32c": [_p, _sz, ctypes.c_uint32],
    "ocrk_edit_distance": [_p, _p, _i32, _p, _p, _i32, _i32, _p, _p, _p],
    "ocrk_conv1_fwd": [_p, _i32, _i32, _i32, _i32, _p, _p, _i32, _p, _i32, _p],
    "ocrk_conv1_wgrad_workspace_size": [_i32, _i32, _i32, _i32],
    "ocrk_conv1_bwd_weight": [_p, _i32, _p, _i32, _i32, _i32, _i32, _p, _p, _i32, _p, _sz, _i32, _p],
    "ocrk_conv2_bwd_data_conv1_wgrad_supported": [_i32, _i32, _i32, _i32, _i32, _i32],
    "ocrk_conv2_bwd_data_conv1_wgrad_workspace_size": [_i32, _i32, _i32],
    "ocrk_conv2_bwd_data_conv1_wgrad": [_p, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p, _p, _i32, _p, _sz, _i32,
                                        _p],
    "ocrk_conv12_bwd_supported": [_i32, _i32, _i32, _i32],
    "ocrk_conv12_bwd_workspace_size": [_i32, _i32, _i32],
    "ocrk_conv12_bwd": [_p, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p, _p, _p, _p, _p, _i32, _p, _sz, _i32, _p],
    "ocrk_conv12_fwd_supported": [_i32, _i32, _i32, _i32],
    "ocrk_conv12_fwd": [_p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _i32, _p],
    "ocrk_conv1_fwd_relu_bits": [_p, _i32, _i32, _i32, _i32, _p, _p, _i32, _p, _p, _i32, _p],
    "ocrk_conv_stats_tiles": [_i64],
    "ocrk_conv3x3_fwd": [_p, _i32, _i32, _i32, _i32, _p, _p, _i32, _p, _i32, _i32, _p, _i32, _p],
    "ocrk_conv3x3_bwd_data_workspace_size": [_i32, _i32, _i32, _i32],
    "ocrk_conv3x3_bwd_data": [_p, _i32, _i32, _i32, _i32, _p, _i32, _p, _p, _p, _i32, _p, _sz, _i32, _p],
    "ocrk_conv3x3_fwd_relu_bits_supported": [_i32, _i32, _i32, _i32, _i32, _i32],
    "ocrk_conv3x3_fwd_relu_bits": [_p, _i32, _i32, _i32, _i32, _p, _p, _i32, _p, _p, _i32, _p],
    "ocrk_conv3x3_bwd_data_bits_supported": [_i32, _i32, _i32, _i32, _i32, _i32],
    "ocrk_conv3x3_bwd_data_bits": [_p, _i32, _i32, _i32, _i32, _p, _i32, _p, _p, _p, _i32, _p, _sz, _i32, _p],
    "ocrk_conv3x3_bwd_data_bits_slab": [_p, _i32, _i32, _i32, _i32, _p, _i32, _p, _p, _p, _i32, _p],
    "ocrk_conv3x3_bwd_data_slab": [_p, _i32, _i32, _i32, _i32, _p, _i32, _p, _p, _p, _i32, _p],
    "ocrk_conv3x3_wgrad_workspace_size": [_i32, _i32, _i32, _i32, _i32],
    "ocrk_conv3x3_bwd_weight": [_p, _p, _i32, _i32, _i32, _i32, _i32, _p, _i32, _p, _sz, _i32, _p],
    "ocrk_bn_finalize_workspace_size": [_i32, _i32],
    "ocrk_bn_finalize": [_p, _i32, _i64, _i32, _f32, _f32, _p, _p, _p, _p, _p, _sz, _p],
    "ocrk_bn_finalize_tiles": [_p, _i32, _i32, _i64, _i32, _f32, _f32, _p, _p, _p, _p, _p, _sz, _p],
    "ocrk_conv3x3_fwd_rowstats_supported": [_i32, _i32, _i32, _i32, _i32],
    "ocrk_conv3x3_fwd_rowstats": [_p, _i32, _i32, _i32, _i32, _p, _p, _i32, _p, _i32, _p, _p],
    "ocrk_bn_infer_params": [_p, _p, _i32, _f32, _p, _p, _p],
    "ocrk_bn_relu_pool_fwd": [_p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _i32, _i32,
                              _p, _i32, _i32, _p],
    "ocrk_bn_bwd_workspace_size": [_i32, _i32, _i32, _i32],
    "ocrk_bn_relu_pool_bwd": [_p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _i32, _i32,
                              _i32, _p, _p, _p, _p, _i32, _p, _sz, _i32, _p],
    "ocrk_bn_moments": [_p, _i32, _i32, _i64, _i32, _p, _p, _sz, _p],
    "ocrk_bn_finalize_moments": [_p, _i32, _f32, _f32, _p, _p, _p, _p, _p],
    "ocrk_bn_bwd_pooled_bias_slab_rows": [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32],
    "ocrk_bn_relu_pool_bwd_pooled": [_p, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _i32, _i32,
                                     _i32, _p, _p, _p, _p, _i32, _p, _p, _sz, _i32, _p],
    "ocrk_bn_relu_pool_bwd_reduce": [_p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _i32, _i32,
                                     _i32, _p, _p, _i32, _p, _p, _sz, _i32, _p],
    "ocrk_bn_relu_pool_bwd_apply": [_p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _i32, _i32,
                                    _i32, _p, _p, _p, _p, _i32, _p, _p, _sz, _i32, _p],
    "ocrk_bn_bwd_bias_slab_rows": [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32],
    "ocrk_bn_relu_pool_bwd_slab": [_p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _i32, _i32,
                                   _i32, _p, _p, _p, _i32, _p, _p, _sz, _i32, _p],
    "ocrk_lstm_fwd_step": [_p, _p, _p, _p, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p],
    "ocrk_lstm_bwd_step": [_p, _p, _p, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p],
    "ocrk_copy_batch": [_p, _i32, _i64, _p],
    "ocrk_gru_fwd_persistent_supported": [_i32, _i32],
    "ocrk_gru_fwd_persistent_workspace_size": [_i32, _i32],
    "ocrk_gru_fwd_persistent": [_p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _sz, _p],
    "ocrk_gru_bwd_persistent_supported": [_i32, _i32],
    "ocrk_gru_bwd_persistent_workspace_size": [_i32, _i32],
    "ocrk_gru_bwd_persistent": [_p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _sz, _p],
    "ocrk_persistent_flags_size": [_i32, _i32],
    "ocrk_lstm_fwd_persistent_supported": [_i32, _i32],
    "ocrk_lstm_fwd_persistent_workspace_size": [_i32, _i32],
    "ocrk_lstm_fwd_persistent": [_p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _sz, _p],
    "ocrk_lstm_fwd_persistent_f32_supported": [_i32, _i32],
    "ocrk_lstm_fwd_persistent_f32_workspace_size": [_i32, _i32],
    "ocrk_lstm_fwd_persistent_f32_flags_size": [_i32, _i32],
    "ocrk_lstm_fwd_persistent_f32": [_p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _sz, _p],
    "ocrk_lstm_bwd_persistent_f32_supported": [_i32, _i32],
    "ocrk_lstm_bwd_persistent_f32_workspace_size": [_i32, _i32],
    "ocrk_lstm_bwd_persistent_f32": [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _sz, _p],
    "ocrk_lstm_bwd_persistent_supported": [_i32, _i32],
    "ocrk_lstm_bwd_persistent_workspace_size": [_i32, _i32],
    "ocrk_lstm_bwd_persistent_slices": [_i32, _i32],
    "ocrk_lstm_bwd_persistent": [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _sz, _p],
    "ocrk_lstm_fwd": [_p, _p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p],
    "ocrk_lstm_bwd": [_p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p],
    "ocrk_gemm_workspace_size": [_i32, _i32, _i32, _i32],
    "ocrk_gemm": [_i32, _i32, _i32, _i32, _i32, _f32, _p, _i64, _i64, _p, _i64, _i64, _p, _i64, _i64,
                  _i32, _p, _i32, _i32, _i32, _i32, _i32, _p, _sz, _p],
    "ocrk_adam": [_p, _p, _p, _p, _i64, _f32, _f32, _f32, _f32, _f32, _p],
    "ocrk_adam_ex": [_p, _p, _p, _p, _i64, _f32, _f32, _f32, _f32, _f32, _u32, _p],
    "ocrk_cast": [_p, _i32, _p, _i32, _i64, _p],
    "ocrk_split_bf16": [_p, _i64, _p, _p, _p],
    "ocrk_permute3": [_p, _i32, _i32, _i32, _i32, _p, _i32, _p],
    "ocrk_strided_copy": [_p, _i64, _i64, _i64, _i64, _p, _i32, _i64, _i64, _p],
    "ocrk_colsum_workspace_size": [_i64, _i32],
    "ocrk_colsum": [_p, _i64, _i32, _i32, _p, _i32, _p, _sz, _p],
    "ocrk_slab_sum_workspace_size": [_i32],
    "ocrk_slab_sum": [_p, _i32, _i32, _i32, _p, _i32, _p, _sz, _p],
    "ocrk_relu_mask": [_p, _p, _i64, _f32, _p, _i32, _p],
    "ocrk_mul_scalar": [_p, _i64, _p, _p],
    "ocrk_mean": [_p, _i32, _p, _p],
    "ocrk_seq_len": [_p, _i32, _p, _p],
    "ocrk_timer_create": [_p],
    "ocrk_timer_record": [_p, _p],
    "ocrk_timer_elapsed": [_p, _p, _p],
    "ocrk_timer_destroy": [_p],
}
_RESTYPE = {"ocrk_last_error": ctypes.c_char_p}
_RESTYPE.update({n: ctypes.c_size_t for n in SIGNATURES if n.endswith("_workspace_size")})
_RESTYPE["ocrk_conv_stats_tiles"] = ctypes.c_size_t
_RESTYPE["ocrk_persistent_flags_size"] = ctypes.c_size_t
_RESTYPE["ocrk_bn_bwd_bias_slab_rows"] = ctypes.c_size_t
_RESTYPE["ocrk_bn_bwd_pooled_bias_slab_rows"] = ctypes.c_size_t
_RESTYPE["ocrk_crc32c"] = ctypes.c_uint32


class OcrkError(RuntimeError):
    """A libocrk entry point returned a non-zero status."""

    def __init__(self, status, message):
        super().__init__(message)
        self.status = status


class InvalidArgumentError(OcrkError):
    """Mirrors tf.errors.InvalidArgumentError (e.g. infeasible CTC labels)."""


class DeviceError(OcrkError):
    """A device-side wait gave up (persistent recurrent kernels): its outputs are invalid."""


# device status word bits (include/ocrk.h, enum ocrk_device_status)
STATUS_CTC_INFEASIBLE = 1 << 1
STATUS_CTC_BAD_LENGTH = 1 << 2
STATUS_CTC_BAD_LABEL = 1 << 3
STATUS_LSTM_FWD_TIMEOUT = 1 << 4
STATUS_LSTM_BWD_TIMEOUT = 1 << 5
STATUS_LSTM_CENSUS = 1 << 6
STATUS_CTC = STATUS_CTC_INFEASIBLE | STATUS_CTC_BAD_LENGTH | STATUS_CTC_BAD_LABEL
STATUS_LSTM = STATUS_LSTM_FWD_TIMEOUT | STATUS_LSTM_BWD_TIMEOUT | STATUS_LSTM_CENSUS

_STATUS_TEXT = {
    STATUS_CTC_INFEASIBLE: "ctc_loss: not enough time for the target transition sequence "
                           "(label + repeats > sequence_length)",
    STATUS_CTC_BAD_LENGTH: "ctc_loss: a label length is negative or exceeds the labels' width",
    STATUS_CTC_BAD_LABEL: "ctc_loss: a label value is outside [0, num_classes - 1)",
    STATUS_LSTM_FWD_TIMEOUT: "persistent recurrent forward: a hand-off wait gave up (co-residency lost)",
    STATUS_LSTM_BWD_TIMEOUT: "persistent recurrent backward: a hand-off wait gave up (co-residency lost)",
    STATUS_LSTM_CENSUS: "persistent recurrent launch: the placement census gave up",
}


# called before a DeviceError is raised for a recurrent-loop status bit
# (kernels.reset_persistent_flags re-zeroes the loops' counting hand-off words)
ON_DEVICE_ERROR = []


def raise_for_status(word):
    """Raise the error a non-zero device status word stands for (CTC bits as
    InvalidArgumentError, like tf.nn.ctc_loss; recurrent timeouts as DeviceError)."""
    word = int(word)
    if not word:
        return
    text = "; ".join(t for b, t in _STATUS_TEXT.items() if word & b)
    if word & STATUS_LSTM:
        for fn in ON_DEVICE_ERROR:
            fn()
        raise DeviceError(OCRK_ERR_HIP, f"device status 0x{word:x}: {text}")
    raise InvalidArgumentError(OCRK_ERR_INFEASIBLE, f"device status 0x{word:x}: {text}")


# include/ocrk_debug.h (exported only by tools/libocrk_exp.so, `make exp`)
DEBUG_SIGNATURES = {
    "ocrk_lstm_debug_stamps": [_p],
    # routes measured slower and kept out of the product library (round 6)
    "ocrk_conv2_bwd_weight_c1x_supported": [_i32, _i32, _i32, _i32],
    "ocrk_conv2_bwd_weight_c1x": [_p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p, _sz, _i32, _p],
    "ocrk_stream_wait": [_p, _p, _i32],
    "ocrk_stream_create_cu_limited": [_i32, _p],
    "ocrk_stream_destroy": [_p],
    "ocrk_lstm_fwd_persistent_x_supported": [_i32, _i32, _i32],
    "ocrk_lstm_fwd_persistent_x": [_p, _i32, _p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _sz, _p],
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make` in the repo root "
                "(or __graft_entry__.build()); there is no CPU fallback")
        handle = ctypes.CDLL(LIB_PATH)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPE.get(name, ctypes.c_int)
        for name, argtypes in DEBUG_SIGNATURES.items():     # include/ocrk_debug.h: tools build only
            if hasattr(handle, name):
                getattr(handle, name).argtypes = argtypes
        _lib = handle
    return _lib


class Timer:
    """A HIP event owned by libocrk (ocrk_timer_*): recorded on torch's current
    stream; inside a hipGraph capture it becomes an external event node, so it
    keeps timestamping on every replay."""

    def __init__(self):
        h = ctypes.c_void_p()
        call("ocrk_timer_create", ctypes.byref(h))
        self.h = h

    def record(self):
        call("ocrk_timer_record", self.h, stream_ptr())

    def elapsed_ms(self, end):
        ms = ctypes.c_float()
        call("ocrk_timer_elapsed", self.h, end.h, ctypes.byref(ms))
        return ms.value

    def __del__(self):
        if _lib is not None and self.h:
            _lib.ocrk_timer_destroy(self.h)


# Optional launch probes (bench.py): name -> (work_fn(args) or None, records list).
# A probed entry point is bracketed by Timers on torch's current stream -- the
# stream every wrapper launches on -- and (start, end, work) is recorded.
PROBES = {}


def call(name, *args):
    """Call ocrk_<name>; raise on a non-zero status."""
    probe = PROBES.get(name)
    if probe is not None and probe[0] is not None and probe[0](args) is None:
        probe = None                                    # the work function filters this launch out
    if probe is not None:
        work_fn, records = probe
        ev0, ev1 = Timer(), Timer()
        ev0.record()
        status = getattr(lib(), name)(*args)
        ev1.record()
        records.append((ev0, ev1, work_fn(args) if work_fn else 0.0))
    else:
        status = getattr(lib(), name)(*args)
    if status != OCRK_OK:
        msg = lib().ocrk_last_error().decode(errors="replace")
        if status in (OCRK_ERR_INFEASIBLE, OCRK_ERR_INVALID_ARG):
            raise InvalidArgumentError(status, msg)
        raise OcrkError(status, msg)
    return status


def ptr(t):
    """Device (or host) address of a tensor, or None for None."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    """The HIP stream handle torch is currently launching on."""
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
