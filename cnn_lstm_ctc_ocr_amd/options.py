"""Engine options: the route and schedule switches kept for A/B measurement and
for the parity tests of alternative routes (no reference counterpart).

Every option starts from its ``OCRK_<NAME>`` environment variable, read ONCE:
the host-side ones here at import, the kernel-side ones by libocrk at its first
launch (``ocrk_get_option`` / ``ocrk_set_option``, include/ocrk.h). After that
only ``set()`` / ``override()`` change them, so no op reads the environment on
its launch path. ``override`` is what tests use to run an alternative route:

    with options.override(LSTM_BWD_R16=0):
        ...                                  # the 32-row gather BPTT
"""
import contextlib
import os

# host-side options (this package) -> default. Round 6 kept only the defaults,
# alternatives that are real routes or documented A/B switches; the routes measured
# slower and kept off (LSTM_FUSE_X, DEFER_BIAS, DEFER_DWX, DX_FIRST, PREFETCH_IMAGES,
# CONV12_RECOMPUTE, CONV_BIAS_SIDE, FORK_EVENTS, SIDE_CU_MASK, TN_ITEMS_LATE, ...) were
# deleted or moved to the tools build (include/ocrk_debug.h); DESIGN.md section 6.
_HOST_DEFAULTS = {
    # real alternatives
    "LSTM_PERSISTENT": 1,     # 0: per-step recurrent kernels instead of the persistent loops
    "F32_TRAIN_EXACT": 0,     # fp32 policy, 1: exact f32 products everywhere (else conv tower only)
    # documented A/B switches (each turns one default route off; the other route stays tested)
    "SIDE_STREAM": 1,         # 0: weight gradients inline on the main stream
    "CONV_SIDE": 1,           # 0: conv weight gradients inline
    "CONV12_FUSED": 1,        # 0: conv1 and conv2 forward as two passes (y1 written, then re-read)
    "RELU_BITS": 1,           # 0: conv3/5/7's ReLU masks for conv4/6/8's backward-data as their bf16 outputs
    "POOLED_BN": 1,           # 0: the BN backward's dgamma / dbeta pass walks z instead of the pooled output
    "CONV1_FUSED": 1,         # 0: conv2's backward-data stores dy1, conv1's weight gradient re-reads it
    "CONV12_BWD": 1,          # 0: conv2's weight gradient as its own launch on y1 (written by the forward)
    # tuning (workgroup caps of the recurrent weight-gradient launches)
    "TN_ITEMS": 256,          # layer 2
    "TN_ITEMS_L1": 160,       # layer 1 (beside the conv backward)
}
# kernel-side options (libocrk's registry, csrc/common.h)
# (LSTM_BWD_KSPLIT, LSTM_BWD_PB16 and PP_DEEP exist in the tools build only)
KERNEL_OPTIONS = ("CONV_DIRECT", "CONV_ROWS", "CONV_ROWS_WIDE", "CONV_WGRAD_BLOCKS", "LSTM_SPIN_LIMIT",
                  "PERSIST_LATE", "LSTM_BWD_R16", "CTC_LDS",
                  "PP_PERSIST_NK", "NT_F32_EXACT", "NT_F32_MASK",
                  "NT_F32_X6", "BEAM_WAVE", "BN_BWD_BLOCKS", "BN_ROUTE", "BN_ROUTE_SEG", "BN_ROUTE_NCH", "CONV_TN_ITEMS", "CONV_TN4_ITEMS",
                  "CONV_WGRAD_CUS", "F32_MFMA", "GEMM_NT", "GEMM_NT_STAGED", "GEMM_PP", "GEMM_PPTN", "PP_MIN_N", "GEMM_TN",
                  "LSTM_DMA", "LSTM_BWD_DMA", "LSTM_FWD_R16", "NT_TAP_UNIFORM")


def _env_int(name, default):
    v = os.environ.get("OCRK_" + name)
    if v is None or v == "":
        return default
    try:
        return int(v)
    except ValueError:
        raise ValueError(f"OCRK_{name}={v!r}: an integer is expected") from None


_HOST = {k: _env_int(k, d) for k, d in _HOST_DEFAULTS.items()}


def get(name):
    """Current value of an option (host-side or kernel-side)."""
    if name in _HOST:
        return _HOST[name]
    if name in KERNEL_OPTIONS:
        import ctypes

        from . import _lib
        v = ctypes.c_int64()
        _lib.call("ocrk_get_option", name.encode(), ctypes.byref(v))
        return v.value
    raise KeyError(f"unknown option {name!r}")


def set(name, value):  # noqa: A001  (module-level setter, options.set)
    """Set an option; returns the previous value."""
    value = int(value)
    if name in _HOST:
        prev, _HOST[name] = _HOST[name], value
        return prev
    if name in KERNEL_OPTIONS:
        import ctypes

        from . import _lib
        prev = ctypes.c_int64()
        _lib.call("ocrk_set_option", name.encode(), value, ctypes.byref(prev))
        return prev.value
    raise KeyError(f"unknown option {name!r}")


@contextlib.contextmanager
def override(**values):
    """Temporarily set options (restored on exit, in reverse order)."""
    prev = []
    try:
        for k, v in values.items():
            prev.append((k, set(k, v)))
        yield
    finally:
        for k, v in reversed(prev):
            set(k, v)
