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

# host-side options (this package) -> default
_HOST_DEFAULTS = {
    "LSTM_PERSISTENT": 1,     # 0: per-step recurrent kernels instead of the persistent loops
    "LSTM_FUSE_X": 0,         # 1: first-layer projection inside the persistent forward (opt-in)
    "BATCHED_IMAGES": 1,      # 0: weight images rebuilt by per-layout copies instead of one batched launch
    "SIDE_STREAM": 1,         # 0: weight gradients inline on the main stream
    "CONV_SIDE": 1,           # 0: conv weight gradients inline
    "DEFER_BIAS": 0,          # 1: bias reductions on their own stream (measured slower)
    "DEFER_DWX": 0,           # 1: an upper layer's dW_x behind the lower BPTT (measured no gain)
    "DX_FIRST": 0,            # 1: the lowest layer's data gradient before its weight gradients
    "PREFETCH_IMAGES": 0,     # 1: the weight-image refresh on its own stream beside conv1 (measured slower)
    "CONV12_FUSED": 1,        # 0: conv1 and conv2 forward as two passes (y1 written, then re-read)
    "CONV12_RECOMPUTE": 0,    # 1: conv12 writes no y1, conv2's weight gradient recomputes it (measured +55 us)
    "CONV_BIAS_SIDE": 0,      # 1: conv / BN bias-gradient reductions ride the next conv side fork (measured slower)
    "CONV_SIDE_MERGE_FROM": 2,  # blocks k > this merge their odd weight gradient into the next fork
    "CONV_SIDE_MERGE": 1,     # 0: a side-stream fork for each conv weight gradient (two per block)
    "RELU_BITS": 1,           # 0: conv3/5/7's ReLU masks for conv4/6/8's backward-data as their bf16 outputs
    "POOLED_BN": 1,           # 0: the BN backward's dgamma / dbeta pass walks z instead of the pooled output
    "CONV1_FUSED": 1,         # 0: conv2's backward-data stores dy1, conv1's weight gradient re-reads it
    "TN_ITEMS": 256,          # workgroup cap of the recurrent weight-gradient launches
    "TN_ITEMS_L1": 160,       # the same for the first layer (beside the conv backward)
    "TN_ITEMS_LATE": 0,       # deferred dW_x cap (0: TN_ITEMS)
    "ADAM_ZERO": 1,           # 0: separate gradient fill instead of the in-Adam zeroing
    "UNIT_SEED": 1,           # 0: backward seeded with torch's ones instead of the resident 1.0
    "FORK_EVENTS": 0,         # 1 / 2: stream forks through ocrk_stream_wait's fence-less events
    "SIDE_CU_MASK": 0,        # > 0: the weight-gradient side stream restricted to this many CUs
    "F32_TRAIN_EXACT": 0,     # 1: fp32 training with exact f32 products everywhere (else conv tower only)
}
# kernel-side options (libocrk's registry, csrc/common.h)
KERNEL_OPTIONS = ("CONV_DIRECT", "CONV_ROWS", "CONV_ROWS_WIDE", "CONV_WGRAD_BLOCKS", "LSTM_SPIN_LIMIT",
                  "PERSIST_LATE", "LSTM_BWD_KSPLIT", "LSTM_BWD_PB16", "LSTM_BWD_R16", "CTC_LDS",
                  "PP_PERSIST_NK", "PP_DEEP", "NT_F32_EXACT", "NT_F32_MASK",
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
if not _HOST["TN_ITEMS_LATE"]:
    _HOST["TN_ITEMS_LATE"] = _HOST["TN_ITEMS"]


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
