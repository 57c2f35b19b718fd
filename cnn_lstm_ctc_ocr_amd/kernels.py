"""Thin torch-tensor wrappers over the libocrk C ABI (one per entry point).

They check shapes/dtypes/devices on the host, allocate outputs and workspaces
with the torch caching allocator, and launch on torch's current stream. They
do no math themselves: every call lands in libocrk.so (include/ocrk.h).
"""
import ctypes

import torch

from . import _lib, options
from ._lib import ptr, call

F32, BF16 = _lib.F32, _lib.BF16
_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dtype_code(dt):
    try:
        return _DT[dt]
    except KeyError:
        raise TypeError(f"unsupported dtype {dt}; libocrk computes in float32 or bfloat16")


def _stream(t):
    return _lib.stream_ptr(t.device)


def _chk(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise ValueError("libocrk ops take device tensors (got a CPU tensor)")
        if not t.is_contiguous():
            raise ValueError("libocrk ops take contiguous tensors")


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# ---------------------------------------------------------------- preprocess
def preprocess(img_u8, dtype=torch.float32):
    """validate._preprocess_image (src/weinman/validate.py:56-68)."""
    if img_u8.dtype != torch.uint8:
        raise TypeError("preprocess expects uint8 pixels")
    _chk(img_u8)
    out = torch.empty(img_u8.shape, dtype=dtype, device=img_u8.device)
    call("ocrk_preprocess", ptr(img_u8), img_u8.numel(), ptr(out), dtype_code(dtype), _stream(img_u8))
    return out


def seq_len(widths):
    """model.py:152-163 on device: floor((w-2)/2) - 2 (int32)."""
    _chk(widths)
    w = widths if widths.dtype == torch.int32 else widths.to(torch.int32)
    out = torch.empty_like(w)
    call("ocrk_seq_len", ptr(w), w.numel(), ptr(out), _stream(w))
    return out


# --------------------------------------------------------------------- conv
def conv1_fwd(x, w, b, dtype, relu_bits=False):
    """x: uint8 [B,H,W] (fused preprocess) or float [B,H,W]; w f32 [3,3,1,C]; -> [B,H-2,W-2,C].
    relu_bits: also return the ReLU's bit mask, u8 [B,H-2,W-2,C/8] (ocrk_conv1_fwd_relu_bits)."""
    _chk(x, w, b)
    B, H, W = x.shape[0], x.shape[1], x.shape[2]
    C = w.shape[-1]
    y = torch.empty(B, H - 2, W - 2, C, dtype=dtype, device=x.device)
    is_u8 = x.dtype == torch.uint8
    if not is_u8 and x.dtype != dtype:
        raise TypeError("conv1 float input must have the compute dtype")
    if relu_bits:
        bits = torch.empty(B, H - 2, W - 2, C // 8, dtype=torch.uint8, device=x.device)
        call("ocrk_conv1_fwd_relu_bits", ptr(x), int(is_u8), B, H, W, ptr(w), ptr(b), C, ptr(y), ptr(bits),
             dtype_code(dtype), _stream(x))
        return y, bits
    call("ocrk_conv1_fwd", ptr(x), int(is_u8), B, H, W, ptr(w), ptr(b), C, ptr(y), dtype_code(dtype), _stream(x))
    return y


def conv12_fwd_ok(x, dtype):
    """The fused conv1 -> conv2 forward covers this image batch [B, IH, IW] (bf16)."""
    B, IH, IW = x.shape[:3]
    return (x.dtype in (torch.uint8, torch.bfloat16) and (x.dtype == torch.uint8 or x.dtype == dtype)
            and bool(_lib.lib().ocrk_conv12_fwd_supported(B, IH, IW, dtype_code(dtype))))


def conv12_fwd(x, w1, b1, w_nk2, b2, want_y1=True):
    """conv1 (fused preprocess, ReLU) -> conv2 (no activation) with conv2's per-row BN
    partials (ocrk_conv12_fwd). Returns y1 [B,IH-2,IW-2,32] bf16 (None unless want_y1:
    the backward recomputes it, conv12_bwd), its ReLU bit mask u8 [.., 4],
    z [B,IH-2,IW-2,32] bf16, stats [B*(IH-2), 2, 32]."""
    _chk(x, w1, b1, w_nk2, b2)
    B, IH, IW = x.shape[:3]
    H, W = IH - 2, IW - 2
    dev = x.device
    y1 = torch.empty(B, H, W, 32, dtype=torch.bfloat16, device=dev) if want_y1 else None
    bits = torch.empty(B, H, W, 4, dtype=torch.uint8, device=dev)
    z = torch.empty(B, H, W, 32, dtype=torch.bfloat16, device=dev)
    stats = torch.empty(B * H, 2, 32, dtype=torch.float32, device=dev)
    call("ocrk_conv12_fwd", ptr(x), int(x.dtype == torch.uint8), B, IH, IW, ptr(w1), ptr(b1), ptr(w_nk2), ptr(b2),
         ptr(y1), ptr(bits), ptr(z), ptr(stats), BF16, _stream(x))
    return y1, bits, z, stats


def conv2_bwd_weight_c1x(x, w1, b1, dz, dw, accumulate=True):
    """conv2's weight gradient with y1 = relu(conv1(x)) recomputed from the image x [B,IH,IW]
    (u8 or bf16) instead of read (ocrk_conv2_bwd_weight_c1x); dz [B,IH-2,IW-2,32] bf16.
    Tools build only (include/ocrk_debug.h): +55 us in the step, not the model's route."""
    _chk(x, w1, b1, dz, dw)
    B, IH, IW = x.shape[:3]
    nb = _lib.lib().ocrk_conv3x3_wgrad_workspace_size(B, IH - 2, IW - 2, 32, 32)
    ws = _ws(nb, x.device)
    call("ocrk_conv2_bwd_weight_c1x", ptr(x), int(x.dtype == torch.uint8), B, IH, IW, ptr(w1), ptr(b1), ptr(dz),
         ptr(dw), int(accumulate), ptr(ws), nb, BF16, _stream(x))


def conv1_bwd_weight(x, dz, dw, db, accumulate=True):
    _chk(x, dz, dw, db)
    B, H, W = x.shape[0], x.shape[1], x.shape[2]
    C = dz.shape[-1]
    nb = _lib.lib().ocrk_conv1_wgrad_workspace_size(B, H, W, C)
    ws = _ws(nb, x.device)
    call("ocrk_conv1_bwd_weight", ptr(x), int(x.dtype == torch.uint8), ptr(dz), B, H, W, C, ptr(dw), ptr(db),
         int(accumulate), ptr(ws), nb, dtype_code(dz.dtype), _stream(x))


def conv2_bwd_data_conv1_wgrad_ok(dz, x):
    """The fused conv2 backward-data + conv1 weight gradient covers this shape
    (bf16, conv2's 32 -> 32 on the row-walking kernel, x u8 or bf16)."""
    B, H, W, C = dz.shape
    return (x.dtype in (torch.uint8, torch.bfloat16) and tuple(x.shape) == (B, H + 2, W + 2)
            and bool(_lib.lib().ocrk_conv2_bwd_data_conv1_wgrad_supported(B, H, W, C, C, dtype_code(dz.dtype))))


def conv2_bwd_data_conv1_wgrad(dz, w_bwd, relu_mask, x, dw, db, accumulate=True, relu_bits=None):
    """dw1 / db1 (+)= conv1's weight / bias gradient, from conv2's pre-BN gradient dz
    through conv2's backward-data and conv1's ReLU (relu_mask = conv1's output, or
    relu_bits = its bit mask from conv1_fwd(..., relu_bits=True) with relu_mask None),
    without storing dy1 (ocrk_conv2_bwd_data_conv1_wgrad)."""
    _chk(dz, w_bwd, relu_mask, relu_bits, x, dw, db)
    if (relu_mask is None) == (relu_bits is None):
        raise ValueError("give exactly one of relu_mask / relu_bits")
    B, H, W, _ = dz.shape
    if relu_bits is not None and (relu_bits.dtype != torch.uint8 or tuple(relu_bits.shape) != (B, H, W, 4)):
        raise ValueError("relu_bits must be uint8 [B, H, W, 4]")
    nb = _lib.lib().ocrk_conv2_bwd_data_conv1_wgrad_workspace_size(B, H, W)
    ws = _ws(nb, dz.device)
    call("ocrk_conv2_bwd_data_conv1_wgrad", ptr(dz), B, H, W, ptr(w_bwd), ptr(relu_mask), ptr(relu_bits), ptr(x),
         int(x.dtype == torch.uint8), ptr(dw), ptr(db), int(accumulate), ptr(ws), nb, dtype_code(dz.dtype),
         _stream(dz))


def conv12_bwd_ok(x, dtype):
    """The fused conv1 -> conv2 backward (ocrk_conv12_bwd) covers this image batch x
    [B, IH, IW] (u8, or bf16 in a bf16 model): dz [B, IH-2, IW-2, 32]."""
    B, IH, IW = x.shape[:3]
    return (x.dim() == 3 and dtype == torch.bfloat16 and x.dtype in (torch.uint8, torch.bfloat16)
            and IH >= 3 and IW >= 3 and bool(_lib.lib().ocrk_conv12_bwd_supported(B, IH - 2, IW - 2, BF16)))


def conv12_bwd(dz, w_bwd, x, w1, b1, dw2, dw1, db1, relu_mask=None, relu_bits=None, accumulate=True):
    """conv2's data and weight gradients and conv1's weight / bias gradients as one row
    walk (ocrk_conv12_bwd): dw2 (+)= conv2's weight gradient with y1 = relu(conv1(x))
    recomputed from the image, dw1 / db1 (+)= conv1's through conv2's backward-data and
    conv1's ReLU (relu_mask = y1, or relu_bits = its bit mask u8 [B, H, W, 4])."""
    _chk(dz, w_bwd, relu_mask, relu_bits, x, w1, b1, dw2, dw1, db1)
    if (relu_mask is None) == (relu_bits is None):
        raise ValueError("give exactly one of relu_mask / relu_bits")
    B, H, W, _ = dz.shape
    if relu_bits is not None and (relu_bits.dtype != torch.uint8 or tuple(relu_bits.shape) != (B, H, W, 4)):
        raise ValueError("relu_bits must be uint8 [B, H, W, 4]")
    nb = _lib.lib().ocrk_conv12_bwd_workspace_size(B, H, W)
    ws = _ws(nb, dz.device)
    call("ocrk_conv12_bwd", ptr(dz), B, H, W, ptr(w_bwd), ptr(relu_mask), ptr(relu_bits), ptr(x),
         int(x.dtype == torch.uint8), ptr(w1), ptr(b1), ptr(dw2), ptr(dw1), ptr(db1), int(accumulate), ptr(ws), nb,
         BF16, _stream(dz))


def conv_stats_tiles(M):
    return _lib.lib().ocrk_conv_stats_tiles(M)


def relu_bits_ok(x_shape, cin, cout, cout_next, dtype):
    """The bit-mask pair covers conv_{odd} (cin -> cout, forward with ReLU) and the next
    conv's (cout -> cout_next) backward-data into it at this [B, H, W] (bf16)."""
    B, H, W = x_shape[:3]
    lib = _lib.lib()
    code = dtype_code(dtype)
    return (bool(lib.ocrk_conv3x3_fwd_relu_bits_supported(B, H, W, cin, cout, code))
            and bool(lib.ocrk_conv3x3_bwd_data_bits_supported(B, H, W, cout_next, cout, code)))


def conv3x3_fwd_relu_bits(x, w_nk, bias):
    """conv3x3_fwd(..., relu=True) and its output's ReLU bit mask, u8 [B, H, W, Cout/8]
    (ocrk_conv3x3_fwd_relu_bits)."""
    _chk(x, w_nk, bias)
    B, H, W, Cin = x.shape
    Cout = w_nk.shape[0]
    y = torch.empty(B, H, W, Cout, dtype=x.dtype, device=x.device)
    bits = torch.empty(B, H, W, Cout // 8, dtype=torch.uint8, device=x.device)
    call("ocrk_conv3x3_fwd_relu_bits", ptr(x), B, H, W, Cin, ptr(w_nk), ptr(bias), Cout, ptr(y), ptr(bits),
         dtype_code(x.dtype), _stream(x))
    return y, bits


def conv3x3_fwd(x, w_nk, bias, relu, stats=None, y_dtype=None):
    _chk(x, w_nk, bias, stats)
    B, H, W, Cin = x.shape
    Cout = w_nk.shape[0]
    y_dtype = y_dtype or x.dtype
    y = torch.empty(B, H, W, Cout, dtype=y_dtype, device=x.device)
    call("ocrk_conv3x3_fwd", ptr(x), B, H, W, Cin, ptr(w_nk), ptr(bias), Cout, ptr(y), dtype_code(y_dtype),
         int(relu), ptr(stats), dtype_code(x.dtype), _stream(x))
    return y


def conv3x3_bwd_data(dy, w_bwd, relu_mask=None, dbias=None, accumulate=True, defer=None, relu_bits=None):
    """dx = conv3x3 backward-data (ReLU mask of the producer fused); if dbias
    is given, dbias (+)= column sums of dx (the producer's bias gradient).
    With a `defer` list, that reduction is appended to it as (fn, tensors) for
    the caller to issue later (e.g. on the side stream): same bits, off the
    data-gradient path (ocrk_conv3x3_bwd_data_slab + ocrk_slab_sum).
    relu_bits (instead of relu_mask): the producer's bit mask from
    conv3x3_fwd_relu_bits (ocrk_conv3x3_bwd_data_bits; no `defer`)."""
    _chk(dy, w_bwd, relu_mask, dbias, relu_bits)
    B, H, W, Cout = dy.shape
    Cin = w_bwd.shape[0]
    dx = torch.empty(B, H, W, Cin, dtype=dy.dtype, device=dy.device)
    if relu_bits is not None:
        if relu_mask is not None:
            raise ValueError("relu_bits replaces relu_mask")
        if dbias is not None and defer is not None:
            tiles = conv_stats_tiles(B * H * W)
            slab = torch.empty(tiles, 2 * Cin, dtype=torch.float32, device=dy.device)
            call("ocrk_conv3x3_bwd_data_bits_slab", ptr(dy), B, H, W, Cout, ptr(w_bwd), Cin, ptr(dx), ptr(relu_bits),
                 ptr(slab), dtype_code(dy.dtype), _stream(dy))
            defer.append((lambda: slab_sum(slab, tiles, Cin, 2 * Cin, dbias, accumulate), (slab,)))
            return dx
        nb, ws = 0, None
        if dbias is not None:
            nb = _lib.lib().ocrk_conv3x3_bwd_data_workspace_size(B, H, W, Cin)
            ws = _ws(nb, dy.device)
        call("ocrk_conv3x3_bwd_data_bits", ptr(dy), B, H, W, Cout, ptr(w_bwd), Cin, ptr(dx), ptr(relu_bits),
             ptr(dbias), int(accumulate), ptr(ws), nb, dtype_code(dy.dtype), _stream(dy))
        return dx
    if dbias is not None and defer is not None:
        tiles = conv_stats_tiles(B * H * W)
        slab = torch.empty(tiles, 2 * Cin, dtype=torch.float32, device=dy.device)
        call("ocrk_conv3x3_bwd_data_slab", ptr(dy), B, H, W, Cout, ptr(w_bwd), Cin, ptr(dx), ptr(relu_mask),
             ptr(slab), dtype_code(dy.dtype), _stream(dy))
        defer.append((lambda: slab_sum(slab, tiles, Cin, 2 * Cin, dbias, accumulate), (slab,)))
        return dx
    nb, ws = 0, None
    if dbias is not None:
        nb = _lib.lib().ocrk_conv3x3_bwd_data_workspace_size(B, H, W, Cin)
        ws = _ws(nb, dy.device)
    call("ocrk_conv3x3_bwd_data", ptr(dy), B, H, W, Cout, ptr(w_bwd), Cin, ptr(dx), ptr(relu_mask), ptr(dbias),
         int(accumulate), ptr(ws), nb, dtype_code(dy.dtype), _stream(dy))
    return dx


def conv3x3_bwd_weight(x, dy, dw, accumulate=True):
    _chk(x, dy, dw)
    B, H, W, Cin = x.shape
    Cout = dy.shape[-1]
    nb = _lib.lib().ocrk_conv3x3_wgrad_workspace_size(B, H, W, Cin, Cout)
    ws = _ws(nb, x.device)
    call("ocrk_conv3x3_bwd_weight", ptr(x), ptr(dy), B, H, W, Cin, Cout, ptr(dw), int(accumulate), ptr(ws), nb,
         dtype_code(x.dtype), _stream(x))


# -------------------------------------------------------------- batch norm
def bn_finalize(stats, M, C, eps, momentum, moving_mean=None, moving_var=None, tile_rows=128):
    """Batch mean / invstd (and the moving averages) from per-tile (sum, M2)
    partials of `tile_rows` rows each (128: the GEMM epilogues; W: the conv2
    row kernel, conv3x3_fwd_rowstats)."""
    _chk(stats, moving_mean, moving_var)
    tiles = stats.shape[0]
    mean = torch.empty(C, dtype=torch.float32, device=stats.device)
    invstd = torch.empty_like(mean)
    nb = _lib.lib().ocrk_bn_finalize_workspace_size(tiles, C)
    ws = _ws(nb, stats.device)
    call("ocrk_bn_finalize_tiles", ptr(stats), tiles, int(tile_rows), M, C, float(eps), float(momentum), ptr(mean),
         ptr(invstd), ptr(moving_mean), ptr(moving_var), ptr(ws), nb, _stream(stats))
    return mean, invstd


def bn_finalize_sync(stats, M, C, eps, momentum, moving_mean, moving_var, tile_rows, group):
    """bn_finalize over the union of the data-parallel ranks' batches (SyncBN):
    this rank's moments [3C + 1] (sum, between-tile and within-tile squares,
    count) SUM-all-reduced over `group`, then finalized; every rank gets the
    same mean / invstd / moving averages. Returns (mean, invstd, count) with
    count the all-reduced pixel total (a device f64 [1], for the backward)."""
    import torch.distributed as dist
    _chk(stats, moving_mean, moving_var)
    tiles = stats.shape[0]
    moments = torch.empty(3 * C + 1, dtype=torch.float64, device=stats.device)
    nb = _lib.lib().ocrk_bn_finalize_workspace_size(tiles, C)
    ws = _ws(nb, stats.device)
    call("ocrk_bn_moments", ptr(stats), tiles, int(tile_rows), M, C, ptr(moments), ptr(ws), nb, _stream(stats))
    dist.all_reduce(moments, op=dist.ReduceOp.SUM, group=group)
    mean = torch.empty(C, dtype=torch.float32, device=stats.device)
    invstd = torch.empty_like(mean)
    call("ocrk_bn_finalize_moments", ptr(moments), C, float(eps), float(momentum), ptr(mean), ptr(invstd),
         ptr(moving_mean), ptr(moving_var), _stream(stats))
    return mean, invstd, moments[3 * C:]


def conv3x3_fwd_rowstats_ok(x, cout):
    """Does the conv2 row kernel take this forward (bf16, Cin = Cout = 32, W <= 254)?"""
    if x.dtype != torch.bfloat16 or not x.is_cuda:
        return False
    B, H, W, cin = x.shape
    return bool(_lib.lib().ocrk_conv3x3_fwd_rowstats_supported(B, H, W, cin, cout))


def conv3x3_fwd_rowstats(x, w_nk, bias, relu=False):
    """(y, stats [B*H, 2, Cout]): the forward with BatchNorm partials per output
    row (finalize with tile_rows = W)."""
    _chk(x, w_nk, bias)
    B, H, W, cin = x.shape
    cout = w_nk.shape[0]
    y = torch.empty(B, H, W, cout, dtype=x.dtype, device=x.device)
    stats = torch.empty(B * H, 2, cout, dtype=torch.float32, device=x.device)
    call("ocrk_conv3x3_fwd_rowstats", ptr(x), B, H, W, cin, ptr(w_nk), ptr(bias), cout, ptr(y), int(relu),
         ptr(stats), _stream(x))
    return y, stats


def bn_infer_params(moving_mean, moving_var, eps):
    _chk(moving_mean, moving_var)
    C = moving_mean.numel()
    mean = torch.empty(C, dtype=torch.float32, device=moving_mean.device)
    invstd = torch.empty_like(mean)
    call("ocrk_bn_infer_params", ptr(moving_mean), ptr(moving_var), C, float(eps), ptr(mean), ptr(invstd),
         _stream(moving_mean))
    return mean, invstd


def bn_relu_pool_fwd(z, mean, invstd, gamma, beta, pool, time_major=False):
    _chk(z, mean, invstd, gamma, beta)
    B, H, W, C = z.shape
    kh, kw, sh, sw = pool
    Ho, Wo = (H - kh) // sh + 1, (W - kw) // sw + 1
    shape = (Wo, B, C) if time_major else (B, Ho, Wo, C)
    out = torch.empty(shape, dtype=z.dtype, device=z.device)
    call("ocrk_bn_relu_pool_fwd", ptr(z), B, H, W, C, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta), kh, kw, sh, sw,
         ptr(out), int(time_major), dtype_code(z.dtype), _stream(z))
    return out


def bn_relu_pool_bwd(z, dp, mean, invstd, gamma, beta, pool, dp_time_major, dgamma, dbeta, accumulate=True,
                     dbias=None, defer=None, sync=None, pooled=None):
    """dz of BN + ReLU + max-pool; dgamma, dbeta and (optionally) dbias = column
    sums of dz (the conv bias in front of the BN) accumulate in f32. With a
    `defer` list the dbias reduction is appended to it as (fn, tensors)
    (ocrk_bn_relu_pool_bwd_slab + ocrk_slab_sum, same bits). sync = (group,
    count): SyncBN -- the batch statistics were bn_finalize_sync's, so the
    backward's two sums are SUM-all-reduced over `group` between its passes.
    pooled: the forward's output (bn_relu_pool_fwd's result, dp's layout) -- the
    dgamma / dbeta pass then streams it and dp instead of walking z
    (ocrk_bn_relu_pool_bwd_pooled; not with sync)."""
    _chk(z, dp, mean, invstd, gamma, beta, dgamma, dbeta, dbias, pooled)
    B, H, W, C = z.shape
    kh, kw, sh, sw = pool
    nb = _lib.lib().ocrk_bn_bwd_workspace_size(B, H, W, C)
    ws = _ws(nb, z.device)
    dz = torch.empty_like(z)
    if sync is not None:
        return _bn_bwd_sync(z, dp, mean, invstd, gamma, beta, pool, dp_time_major, dgamma, dbeta, accumulate, dbias,
                            defer, sync, dz, ws, nb)
    if pooled is not None:
        if pooled.shape != dp.shape or pooled.dtype != dp.dtype:
            raise ValueError("pooled must have dp's shape and dtype")
        # 0 rows: the library takes the z form for this pool (or BN_ROUTE=0) -- use it here too,
        # so a deferred bias slab has the z form's C-wide rows
        rows = _lib.lib().ocrk_bn_bwd_pooled_bias_slab_rows(B, H, W, C, kh, kw, sh, sw)
        if rows == 0:
            pooled = None
    if pooled is not None:
        slab = None
        if dbias is not None and defer is not None:
            # [bias | dgamma] partial rows: both reductions deferred
            slab = torch.empty(rows, 2 * C, dtype=torch.float32, device=z.device)
        call("ocrk_bn_relu_pool_bwd_pooled", ptr(z), ptr(pooled), ptr(dp), B, H, W, C, ptr(mean), ptr(invstd),
             ptr(gamma), ptr(beta), kh, kw, sh, sw, int(dp_time_major), ptr(dz), ptr(dgamma), ptr(dbeta),
             ptr(dbias), int(accumulate), ptr(slab), ptr(ws), nb, dtype_code(z.dtype), _stream(z))
        if slab is not None:
            def _late():
                slab_sum(slab, rows, C, 2 * C, dbias, accumulate)
                slab_sum(slab.view(-1)[C:], rows, C, 2 * C, dgamma, accumulate)
            defer.append((_late, (slab,)))
        return dz
    if dbias is not None and defer is not None:
        rows = _lib.lib().ocrk_bn_bwd_bias_slab_rows(B, H, W, C, kh, kw, sh, sw)
        slab = torch.empty(rows, C, dtype=torch.float32, device=z.device)
        call("ocrk_bn_relu_pool_bwd_slab", ptr(z), ptr(dp), B, H, W, C, ptr(mean), ptr(invstd), ptr(gamma),
             ptr(beta), kh, kw, sh, sw, int(dp_time_major), ptr(dz), ptr(dgamma), ptr(dbeta), int(accumulate),
             ptr(slab), ptr(ws), nb, dtype_code(z.dtype), _stream(z))
        defer.append((lambda: slab_sum(slab, rows, C, C, dbias, accumulate), (slab,)))
        return dz
    call("ocrk_bn_relu_pool_bwd", ptr(z), ptr(dp), B, H, W, C, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta),
         kh, kw, sh, sw, int(dp_time_major), ptr(dz), ptr(dgamma), ptr(dbeta), ptr(dbias), int(accumulate),
         ptr(ws), nb,
         dtype_code(z.dtype), _stream(z))
    return dz


def _bn_bwd_sync(z, dp, mean, invstd, gamma, beta, pool, dp_time_major, dgamma, dbeta, accumulate, dbias, defer,
                 sync, dz, ws, nb):
    import torch.distributed as dist
    group, count = sync
    B, H, W, C = z.shape
    kh, kw, sh, sw = pool
    dsum = torch.empty(2 * C, dtype=torch.float32, device=z.device)
    args = (ptr(z), ptr(dp), B, H, W, C, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta), kh, kw, sh, sw,
            int(dp_time_major))
    call("ocrk_bn_relu_pool_bwd_reduce", *args, ptr(dgamma), ptr(dbeta), int(accumulate), ptr(dsum), ptr(ws), nb,
         dtype_code(z.dtype), _stream(z))
    dist.all_reduce(dsum, op=dist.ReduceOp.SUM, group=group)
    slab = None
    if dbias is not None and defer is not None:
        rows = _lib.lib().ocrk_bn_bwd_bias_slab_rows(B, H, W, C, kh, kw, sh, sw)
        slab = torch.empty(rows, C, dtype=torch.float32, device=z.device)
    call("ocrk_bn_relu_pool_bwd_apply", *args, ptr(dsum), ptr(count), ptr(dz),
         ptr(dbias if slab is None else None), int(accumulate), ptr(slab), ptr(ws), nb, dtype_code(z.dtype), _stream(z))
    if slab is not None:
        defer.append((lambda: slab_sum(slab, rows, C, C, dbias, accumulate), (slab,)))
    return dz


# ---------------------------------------------------------------- GEMM
def gemm(a, b, trans_a=False, trans_b=False, bias=None, relu=False, out=None, out_dtype=torch.float32,
         accumulate=False, alpha=1.0, M=None, N=None, K=None, lda=None, ldb=None, ldc=None,
         batch=1, stride_a=0, stride_b=0, stride_c=0, splits=1):
    """C = alpha op(A) op(B) (+bias) (relu) (+= C). A, B contiguous 2-D unless explicit
    sizes/leading dimensions are given (then they may be strided views)."""
    for t in (a, b, bias, out):
        if t is not None and not t.is_cuda:
            raise ValueError("libocrk ops take device tensors (got a CPU tensor)")
    if M is None:
        _chk(a, b)
        M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
        N = b.shape[0] if trans_b else b.shape[1]
        lda, ldb = a.shape[1], b.shape[1]
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=a.device)
        ldc = N
    ldc = ldc if ldc is not None else N
    if a.dtype != b.dtype:
        raise TypeError("gemm operands must share a dtype")
    kc = -(-(-(-K // splits)) // 32) * 32 if splits > 1 else K
    splits = -(-K // kc) if splits > 1 else 1
    nb = _lib.lib().ocrk_gemm_workspace_size(M, N, batch, splits) if splits > 1 else 0
    ws = _ws(nb, a.device) if nb else None
    call("ocrk_gemm", int(trans_a), int(trans_b), M, N, K, float(alpha), ptr(a), lda, stride_a, ptr(b), ldb,
         stride_b, ptr(out), ldc, stride_c, dtype_code(out.dtype), ptr(bias), int(relu), int(accumulate),
         batch, dtype_code(a.dtype), splits, ptr(ws), nb, _stream(a))
    return out


# ------------------------------------------------------------------ LSTM
_PERSISTENT = {}


def lstm_persistent_ok(B, H, dtype):
    """Run the bf16 time loops as persistent launches (csrc/lstm_persistent.hip)?
    On by default where the grid fits co-resident (B % 32 == 0, H in {256,
    512}); OCRK_LSTM_PERSISTENT=0 selects the per-step kernels."""
    if dtype != torch.bfloat16 or not options.get("LSTM_PERSISTENT"):
        return False
    key = (B, H)
    if key not in _PERSISTENT:
        lib = _lib.lib()
        _PERSISTENT[key] = bool(lib.ocrk_lstm_fwd_persistent_supported(B, H)) and \
            bool(lib.ocrk_lstm_bwd_persistent_supported(B, H))
    return _PERSISTENT[key]


_STATUS = {}
_FLAGS = {}


def persistent_flags(kind, B, H, device, size_fn="ocrk_persistent_flags_size"):
    """The counting hand-off words of one persistent entry point (include/ocrk.h,
    ocrk_persistent_flags_size): zeroed once per (entry point, B, H, device,
    stream) and kept, so the loops need no clearing launch in front of them.
    Launches on one stream never overlap, so they may share it; a hipGraph
    replay keeps counting in the buffer it captured."""
    device = torch.device(device)
    key = (kind, B, H, device, torch.cuda.current_stream(device).cuda_stream)
    t = _FLAGS.get(key)
    if t is None:
        nb = getattr(_lib.lib(), size_fn)(B, H)
        t = _FLAGS[key] = torch.zeros(max(int(nb), 16) // 4, dtype=torch.int32, device=device)
    return t


def reset_persistent_flags():
    """Re-zero every kept hand-off buffer after a device error. Defensive: every
    member of a loop that gave up still posts all of its flags, so the counts
    stay equal; but a kernel that faulted or was killed mid-loop would leave
    them unequal, and the next launch's base would be wrong. In place, so
    captured graphs stay valid; each owning device is synchronised."""
    for t in _FLAGS.values():
        t.zero_()
    for d in {t.device for t in _FLAGS.values()}:
        torch.cuda.synchronize(d)


_lib.ON_DEVICE_ERROR.append(reset_persistent_flags)


def status_word(device):
    """The device status word (include/ocrk.h, ocrk_device_status): one u32 per
    device that the CTC kernel and the persistent recurrent kernels OR their
    failure bits into. Read it at a sync point with check_status / read_status."""
    device = torch.device(device)
    if device not in _STATUS:
        _STATUS[device] = torch.zeros(1, dtype=torch.int32, device=device)
    return _STATUS[device]


lstm_error_word = status_word          # the persistent kernels' bits live in the same word


def clear_status(device, bits):
    """Clear exactly `bits` of the device status word (stream-ordered atomic
    AND-NOT, ocrk_status_clear): bits set meanwhile by in-flight launches stay."""
    w = status_word(device)
    if bits:
        call("ocrk_status_clear", ptr(w), int(bits) & 0xFFFFFFFF, _stream(w))


def read_status(device, reset=True):
    """Synchronising read of the device status word (the bits read are cleared
    when reset)."""
    w = status_word(device)
    v = int(w.item())
    if v and reset:
        clear_status(device, v)
    return v


def check_status(device, reset=True):
    """Raise (InvalidArgumentError / DeviceError) if the device status word is set."""
    _lib.raise_for_status(read_status(device, reset))


class f32_exact:
    """Context manager: fp32 GEMMs / convs with exact f32 MFMA products while
    inside (ocrk_set_f32_gemm_mode(1)), and the fp32 recurrence on the per-step
    f32 kernels; the default outside is the bf16x3 split (include/ocrk.h).
    Process-wide (the autograd engine runs a backward's launches on its own
    device thread, which must see the mode): serving launched from another
    thread while a training step is inside runs exact fp32 products as well
    (still fp32-correct, slower); INTEGRATION.md "precision"."""

    def __init__(self, on=True):
        self.on = on
        self.prev = None

    def __enter__(self):
        self.prev = _lib.lib().ocrk_set_f32_gemm_mode(1 if self.on else 0)
        return self

    def __exit__(self, *exc):
        _lib.lib().ocrk_set_f32_gemm_mode(self.prev)
        return False


def f32_mode_exact():
    return bool(_lib.lib().ocrk_f32_gemm_exact())


def lstm_f32_persistent_ok(B, H):
    """Run the fp32 forward loop as one persistent launch on the bf16x3 split
    (csrc/lstm_f32x3.hip)? H = 512, B % 16 == 0 and the grid co-resident; not
    in exact fp32 mode (f32_exact); OCRK_LSTM_PERSISTENT=0 selects the per-step
    fp32 kernels."""
    if not options.get("LSTM_PERSISTENT") or f32_mode_exact():
        return False
    key = ("f32", B, H)
    if key not in _PERSISTENT:
        _PERSISTENT[key] = bool(_lib.lib().ocrk_lstm_fwd_persistent_f32_supported(B, H))
    return _PERSISTENT[key]


def lstm_f32_bwd_persistent_ok(B, H):
    """Run the fp32 BPTT as one persistent launch on the bf16x3 split
    (csrc/lstm_f32x3.hip)? H = 512, B % 32 == 0 and the B-workgroup grid
    co-resident; not in exact fp32 mode; OCRK_LSTM_PERSISTENT=0 selects the
    per-step fp32 kernels."""
    if not options.get("LSTM_PERSISTENT") or f32_mode_exact():
        return False
    key = ("f32bwd", B, H)
    if key not in _PERSISTENT:
        _PERSISTENT[key] = bool(_lib.lib().ocrk_lstm_bwd_persistent_f32_supported(B, H))
    return _PERSISTENT[key]


def lstm_fwd(gx, whT, seq_len, T, B, H, dtype, save=True):
    """One bidirectional LSTM layer's time loop. Returns (out, hprev, cprev, acts);
    save=False (no backward will run): the fp32 persistent loop skips the saved
    tensors and returns None for them."""
    _chk(gx, whT, seq_len)
    if gx.dtype != dtype or whT.dtype != dtype:
        raise TypeError(f"lstm_fwd: gx and whT must be {dtype} (got {gx.dtype}, {whT.dtype})")
    dev = gx.device
    if dtype == torch.float32 and lstm_f32_persistent_ok(B, H):
        out = torch.empty(T, B, 2 * H, dtype=dtype, device=dev)       # padded steps written as zeros by the kernel
        hprev = cprev = acts = None
        if save:
            hprev = torch.empty(T, B, 2, H, dtype=dtype, device=dev)
            cprev = torch.empty(T, B, 2, H, dtype=torch.float32, device=dev)
            acts = torch.empty(T, B, 2, 4 * H, dtype=dtype, device=dev)
        nb = _lib.lib().ocrk_lstm_fwd_persistent_f32_workspace_size(B, H)
        ws = _ws(nb, dev)
        call("ocrk_lstm_fwd_persistent_f32", ptr(gx), ptr(whT), ptr(seq_len), T, B, H, ptr(out), ptr(hprev),
             ptr(cprev), ptr(acts), ptr(lstm_error_word(dev)),
             ptr(persistent_flags("lstm_fwd_f32", B, H, dev, "ocrk_lstm_fwd_persistent_f32_flags_size")),
             ptr(ws), nb, _stream(gx))
        return out, hprev, cprev, acts
    if lstm_persistent_ok(B, H, dtype):
        out = torch.empty(T, B, 2 * H, dtype=dtype, device=dev)       # padded steps written as zeros by the kernel
        hprev = torch.empty(T, B, 2, H, dtype=dtype, device=dev)
        cprev = torch.empty(T, B, 2, H, dtype=torch.float32, device=dev)
        acts = torch.empty(T, B, 2, 4 * H, dtype=dtype, device=dev)
        nb = _lib.lib().ocrk_lstm_fwd_persistent_workspace_size(B, H)
        ws = _ws(nb, dev)
        call("ocrk_lstm_fwd_persistent", ptr(gx), ptr(whT), ptr(seq_len), T, B, H, ptr(out), ptr(hprev),
             ptr(cprev), ptr(acts), ptr(lstm_error_word(dev)), ptr(persistent_flags("lstm_fwd", B, H, dev)), ptr(ws),
             nb, _stream(gx))
        return out, hprev, cprev, acts
    h_state = torch.zeros(2, 2, B, H, dtype=dtype, device=dev)
    c_state = torch.zeros(2, B, H, dtype=torch.float32, device=dev)
    out = torch.zeros(T, B, 2 * H, dtype=dtype, device=dev)
    hprev = torch.empty(T, B, 2, H, dtype=dtype, device=dev)
    cprev = torch.empty(T, B, 2, H, dtype=torch.float32, device=dev)
    acts = torch.empty(T, B, 2, 4 * H, dtype=dtype, device=dev)
    call("ocrk_lstm_fwd", ptr(gx), ptr(whT), ptr(h_state), ptr(c_state), ptr(seq_len), T, B, H, ptr(out),
         ptr(hprev), ptr(cprev), ptr(acts), dtype_code(dtype), _stream(gx))
    return out, hprev, cprev, acts


def lstm_fused_x_ok(B, H, n_in, dtype):
    """Can the tools build (include/ocrk_debug.h) run the first layer's input
    projection fused into the persistent forward (ocrk_lstm_fwd_persistent_x)?
    Never the model's route: measured at B=256 it removes the 109 us projection
    GEMM but makes every step 0.7 us longer (3.40 vs 2.68 us: the x.W_x MFMAs and
    the x-row DMA land on the step's critical path), 480 vs 490 us for GEMM +
    loop alone and 5.865 vs 5.847 ms for the train step
    (profiles/r3_fused_projection.txt)."""
    if not lstm_persistent_ok(B, H, dtype) or not hasattr(_lib.lib(), "ocrk_lstm_fwd_persistent_x_supported"):
        return False
    return bool(_lib.lib().ocrk_lstm_fwd_persistent_x_supported(B, H, n_in))


def lstm_fwd_fused_x(x, wxT, bias, whT, seq_len, T, B, H):
    """The persistent forward with x . W_x + b fused (no gx): x [T,B,In] bf16,
    wxT [8H, In] (fw | bw W_x^T), bias f32 [8H]. Same outputs as lstm_fwd."""
    _chk(x, wxT, bias, whT, seq_len)
    dev = x.device
    n_in = x.shape[-1]
    out = torch.empty(T, B, 2 * H, dtype=x.dtype, device=dev)
    hprev = torch.empty(T, B, 2, H, dtype=x.dtype, device=dev)
    cprev = torch.empty(T, B, 2, H, dtype=torch.float32, device=dev)
    acts = torch.empty(T, B, 2, 4 * H, dtype=x.dtype, device=dev)
    nb = _lib.lib().ocrk_lstm_fwd_persistent_workspace_size(B, H)
    ws = _ws(nb, dev)
    call("ocrk_lstm_fwd_persistent_x", ptr(x), n_in, ptr(wxT), ptr(bias), ptr(whT), ptr(seq_len), T, B, H, ptr(out),
         ptr(hprev), ptr(cprev), ptr(acts), ptr(lstm_error_word(dev)), ptr(persistent_flags("lstm_fwd_x", B, H, dev)),
         ptr(ws), nb, _stream(x))
    return out, hprev, cprev, acts


def lstm_bwd(wh, seq_len, dout, cprev, acts, T, B, H, dbias=None, defer=None):
    """dG [T,B,2,4H]. dbias (f32 [2*4H], accumulated): the layer's bias gradient
    (both directions); the persistent loop forms it in-kernel (per-slice
    partials, summed by ocrk_slab_sum -- appended to `defer` as (fn, tensors)
    when given), the per-step path by a column sum of dG."""
    _chk(wh, seq_len, dout, cprev, acts, dbias)
    dtype = dout.dtype
    dev = dout.device
    dG = torch.empty(T, B, 2, 4 * H, dtype=dtype, device=dev)
    if dtype == torch.float32 and lstm_f32_bwd_persistent_ok(B, H):
        nb = _lib.lib().ocrk_lstm_bwd_persistent_f32_workspace_size(B, H)
        ws = _ws(nb, dev)
        part = torch.empty(B // 32, 2 * 4 * H, dtype=torch.float32, device=dev) if dbias is not None else None
        call("ocrk_lstm_bwd_persistent_f32", ptr(wh), ptr(seq_len), T, B, H, ptr(dout), ptr(cprev), ptr(acts),
             ptr(dG), ptr(lstm_error_word(dev)), ptr(persistent_flags("lstm_bwd_f32", B, H, dev)), ptr(part),
             ptr(ws), nb, _stream(dout))
        if dbias is not None:
            _bias_parts(part, B // 32, 2 * 4 * H, dbias, defer)
        return dG
    if lstm_persistent_ok(B, H, dtype):
        nb = _lib.lib().ocrk_lstm_bwd_persistent_workspace_size(B, H)
        ws = _ws(nb, dev)
        slices = _lib.lib().ocrk_lstm_bwd_persistent_slices(B, H)     # B/16 (16-row members) or B/32
        part = torch.empty(slices, 2 * 4 * H, dtype=torch.float32, device=dev) if dbias is not None else None
        call("ocrk_lstm_bwd_persistent", ptr(wh), ptr(seq_len), T, B, H, ptr(dout), ptr(cprev), ptr(acts), ptr(dG),
             ptr(lstm_error_word(dev)), ptr(persistent_flags("lstm_bwd", B, H, dev)), ptr(part), ptr(ws), nb,
             _stream(dout))
        if dbias is not None:
            _bias_parts(part, slices, 2 * 4 * H, dbias, defer)
        return dG
    dg_state = torch.zeros(2, 2, B, 4 * H, dtype=dtype, device=dev)
    dc_state = torch.zeros(2, B, H, dtype=torch.float32, device=dev)
    call("ocrk_lstm_bwd", ptr(wh), ptr(dg_state), ptr(dc_state), ptr(seq_len), T, B, H, ptr(dout), ptr(cprev),
         ptr(acts), ptr(dG), dtype_code(dtype), _stream(dout))
    if dbias is not None:
        colsum(dG, T * B, 2 * 4 * H, dbias)
    return dG


# ------------------------------------------------------------------- GRU
_GRU_PERSISTENT = {}


def gru_persistent_ok(B, H, dtype):
    """Run the bf16 GRU time loops as persistent launches (csrc/gru_persistent.hip)?
    Same rule and switch as the LSTM: B % 32 == 0, H in {256, 512}, the grid
    co-resident; OCRK_LSTM_PERSISTENT=0 selects the per-step kernels."""
    if dtype != torch.bfloat16 or not options.get("LSTM_PERSISTENT"):
        return False
    key = (B, H)
    if key not in _GRU_PERSISTENT:
        lib = _lib.lib()
        _GRU_PERSISTENT[key] = bool(lib.ocrk_gru_fwd_persistent_supported(B, H)) and \
            bool(lib.ocrk_gru_bwd_persistent_supported(B, H))
    return _GRU_PERSISTENT[key]


def gru_fwd(gx, whgT, whcT, seq_len, T, B, H, dtype):
    """Returns out [T,B,2H], hprev_t, rh_t [T,B,2,H], acts_t [T,B,2,3H] (dtype)."""
    _chk(gx, whgT, whcT, seq_len)
    if gx.dtype != dtype or whgT.dtype != dtype:
        raise TypeError(f"gru_fwd: gx and weights must be {dtype} (got {gx.dtype}, {whgT.dtype})")
    dev = gx.device
    if gru_persistent_ok(B, H, dtype):
        out = torch.empty(T, B, 2 * H, dtype=dtype, device=dev)       # padded steps written as zeros by the kernel
        hprev = torch.empty(T, B, 2, H, dtype=dtype, device=dev)
        rh_t = torch.empty(T, B, 2, H, dtype=dtype, device=dev)
        acts = torch.empty(T, B, 2, 3 * H, dtype=dtype, device=dev)
        nb = _lib.lib().ocrk_gru_fwd_persistent_workspace_size(B, H)
        ws = _ws(nb, dev)
        call("ocrk_gru_fwd_persistent", ptr(gx), ptr(whgT), ptr(whcT), ptr(seq_len), T, B, H, ptr(out), ptr(hprev),
             ptr(rh_t), ptr(acts), ptr(status_word(dev)), ptr(persistent_flags("gru_fwd", B, H, dev)), ptr(ws), nb,
             _stream(gx))
        return out, hprev, rh_t, acts
    h = torch.zeros(2, B, H, dtype=dtype, device=dev)
    rh = torch.empty(2, B, H, dtype=dtype, device=dev)
    out = torch.zeros(T, B, 2 * H, dtype=dtype, device=dev)
    hprev = torch.empty(T, B, 2, H, dtype=dtype, device=dev)
    rh_t = torch.empty(T, B, 2, H, dtype=dtype, device=dev)
    acts = torch.empty(T, B, 2, 3 * H, dtype=dtype, device=dev)
    call("ocrk_gru_fwd", ptr(gx), ptr(whgT), ptr(whcT), ptr(h), ptr(rh), ptr(seq_len), T, B, H, ptr(out),
         ptr(hprev), ptr(rh_t), ptr(acts), dtype_code(dtype), _stream(gx))
    return out, hprev, rh_t, acts


def gru_bwd(whg, whc, seq_len, dout, hprev, acts, T, B, H, dbias=None, defer=None):
    """Returns dG_t [T,B,2,3H] = (dz_r, dz_u, dz_c) per direction. dbias (f32
    [2*3H], accumulated): the layer's [gates | candidate] bias gradients, formed
    in the persistent loop (else a column sum of dG)."""
    _chk(whg, whc, seq_len, dout, hprev, acts, dbias)
    dtype = dout.dtype
    dev = dout.device
    if gru_persistent_ok(B, H, dtype):
        dG = torch.empty(T, B, 2, 3 * H, dtype=dtype, device=dev)
        nb = _lib.lib().ocrk_gru_bwd_persistent_workspace_size(B, H)
        ws = _ws(nb, dev)
        part = torch.empty(B // 32, 2 * 3 * H, dtype=torch.float32, device=dev) if dbias is not None else None
        call("ocrk_gru_bwd_persistent", ptr(whg), ptr(whc), ptr(seq_len), T, B, H, ptr(dout), ptr(hprev), ptr(acts),
             ptr(dG), ptr(status_word(dev)), ptr(persistent_flags("gru_bwd", B, H, dev)), ptr(part), ptr(ws), nb,
             _stream(dout))
        if dbias is not None:
            _bias_parts(part, B // 32, 2 * 3 * H, dbias, defer)
        return dG
    dzg = torch.empty(2, B, 2 * H, dtype=dtype, device=dev)
    dzc = torch.empty(2, B, H, dtype=dtype, device=dev)
    dh_tot = torch.empty(2, B, H, dtype=torch.float32, device=dev)
    direct = torch.empty(2, B, H, dtype=torch.float32, device=dev)
    dG = torch.empty(T, B, 2, 3 * H, dtype=dtype, device=dev)
    call("ocrk_gru_bwd", ptr(whg), ptr(whc), ptr(dzg), ptr(dzc), ptr(dh_tot), ptr(direct), ptr(seq_len), T, B, H,
         ptr(dout), ptr(hprev), ptr(acts), ptr(dG), dtype_code(dtype), _stream(dout))
    if dbias is not None:
        colsum(dG, T * B, 2 * 3 * H, dbias)
    return dG


# ----------------------------------------------------------------- misc
def split_bf16(x):
    """(hi, lo) bf16 planes of an fp32 tensor: x = hi + lo to 2^-17 (ocrk_split_bf16)."""
    _chk(x)
    if x.dtype != torch.float32 or not x.is_contiguous():
        raise TypeError("split_bf16 takes a contiguous float32 tensor")
    hi = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    lo = torch.empty_like(hi)
    call("ocrk_split_bf16", ptr(x), x.numel(), ptr(hi), ptr(lo), _stream(x))
    return hi, lo


def split_products(*tensors):
    """Operand sets for an fp32 product on the bf16 engines through the split:
    [(a_hi, b_hi, ...), (a_hi, b_lo), (a_lo, b_hi)] for two operands (the al.bl
    term, ~2^-18 relative, is dropped -- mfma_util.h split2_bf16)."""
    a, b = (split_bf16(t) for t in tensors)
    return [(a[0], b[0]), (a[0], b[1]), (a[1], b[0])]


def cast(x, dtype, out=None):
    _chk(x)
    out = out if out is not None else torch.empty(x.shape, dtype=dtype, device=x.device)
    call("ocrk_cast", ptr(x), dtype_code(x.dtype), ptr(out), dtype_code(out.dtype), x.numel(), _stream(x))
    return out


def permute3(x, d0, d1, d2, dtype, out=None):
    _chk(x)
    out = out if out is not None else torch.empty(d1, d0, d2, dtype=dtype, device=x.device)
    call("ocrk_permute3", ptr(x), dtype_code(x.dtype), d0, d1, d2, ptr(out), dtype_code(out.dtype), _stream(x))
    return out


def stream_wait(waiter, signaller, mode=1):
    """`waiter` (a torch.cuda.Stream) waits for the work issued so far on
    `signaller` (ocrk_stream_wait: an event without the system-scope release).
    Tools build only (include/ocrk_debug.h, OCRK_LIB=tools/libocrk_exp.so): the
    fence-less forks measured box-dependent (-35 to +25 us per step)."""
    call("ocrk_stream_wait", ctypes.c_void_p(waiter.cuda_stream), ctypes.c_void_p(signaller.cuda_stream), int(mode))


_CU_STREAMS = []        # (handle, ExternalStream): kept for the process


def cu_limited_stream(device, n_cus):
    """torch.cuda.ExternalStream over ocrk_stream_create_cu_limited(n_cus) on `device`
    (tools build only). A BLOCKING stream: beside a step on the legacy NULL stream it
    serialises with it; beside a non-blocking step stream masks of 96-192 CUs measured
    no change (profiles/r6_stream_ab.txt)."""
    with torch.cuda.device(device):
        h = ctypes.c_void_p()
        call("ocrk_stream_create_cu_limited", int(n_cus), ctypes.byref(h))
        st = torch.cuda.ExternalStream(h.value, device=device)
    _CU_STREAMS.append((h, st))
    return st


def fork(waiter, signaller):
    """waiter.wait_stream(signaller): the step's cross-stream forks (torch events)."""
    waiter.wait_stream(signaller)


def wait_mark(waiter, mark):
    """waiter waits for a pending entry (a torch.cuda.Event)."""
    waiter.wait_event(mark)


def copy_batch(table, njobs, total_tiles, stream_of):
    """One launch of the 2-D copy jobs in `table` (int64 device tensor [njobs, 8],
    include/ocrk.h ocrk_copy_batch): the weight images of a parameter version."""
    _chk(table, stream_of)
    call("ocrk_copy_batch", ptr(table), int(njobs), int(total_tiles), _stream(stream_of))


def strided_copy(src, rows, cols, in_rs, in_cs, out, out_rs, out_cs, out_offset=0, in_offset=0):
    """out.flat[out_offset + r*out_rs + c*out_cs] = src.flat[in_offset + r*in_rs + c*in_cs]."""
    _chk(src, out)
    sp = ctypes_offset(src, in_offset)
    op = ctypes_offset(out, out_offset)
    call("ocrk_strided_copy", sp, rows, cols, in_rs, in_cs, op, dtype_code(out.dtype), out_rs, out_cs, _stream(src))


def ctypes_offset(t, elems):
    return ctypes.c_void_p(t.data_ptr() + elems * t.element_size())


def slab_sum(slab, nslab, nc, ld, out, accumulate=True):
    """out[:nc] (+)= the column sums of slab [nslab][ld] f32 (fixed order, double accumulation)."""
    _chk(slab, out)
    nb = _lib.lib().ocrk_slab_sum_workspace_size(nc)
    ws = _ws(nb, slab.device)
    call("ocrk_slab_sum", ptr(slab), int(nslab), int(nc), int(ld), ptr(out), int(accumulate), ptr(ws), nb,
         _stream(slab))


def _bias_parts(part, rows, nc, dbias, defer):
    if defer is None:
        slab_sum(part, rows, nc, nc, dbias)
    else:
        defer.append((lambda: slab_sum(part, rows, nc, nc, dbias), (part,)))


def colsum(x, M, N, out, accumulate=True):
    _chk(x, out)
    nb = _lib.lib().ocrk_colsum_workspace_size(M, N)
    ws = _ws(nb, x.device)
    call("ocrk_colsum", ptr(x), M, N, dtype_code(x.dtype), ptr(out), int(accumulate), ptr(ws), nb, _stream(x))


def relu_mask(dy, y, out_dtype, scale=1.0):
    _chk(dy, y)
    out = torch.empty(dy.shape, dtype=out_dtype, device=dy.device)
    call("ocrk_relu_mask", ptr(dy), ptr(y), dy.numel(), float(scale), ptr(out), dtype_code(out_dtype), _stream(dy))
    return out


def mul_scalar_(x, s):
    _chk(x, s)
    call("ocrk_mul_scalar", ptr(x), x.numel(), ptr(s), _stream(x))
    return x


def mean(x):
    _chk(x)
    out = torch.empty((), dtype=torch.float32, device=x.device)
    call("ocrk_mean", ptr(x), x.numel(), ptr(out), _stream(x))
    return out


def adam_(p, g, m, v, lr_t, beta1=0.9, beta2=0.999, eps=1e-8, grad_scale=1.0, zero_grad=False):
    """zero_grad: g is cleared as it is read (OCRK_ADAM_ZERO_GRAD)."""
    _chk(p, g, m, v)
    call("ocrk_adam_ex", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), float(lr_t), float(beta1), float(beta2),
         float(eps), float(grad_scale), 1 if zero_grad else 0, _stream(p))


# ----------------------------------------------------------------------- CTC
def ctc_loss(logits, labels, label_len, seq_len, grad_scale=1.0, need_grad=True, status=None):
    """Per-sequence CTC loss (and grad_scale * dloss/dlogits).

    logits f32 [T,B,C]; labels i32 [B,Lmax]; label_len, seq_len i32 [B].
    Returns (loss [B], grad [T,B,C] or None, status i32 [B])."""
    if logits.dtype != torch.float32:
        raise TypeError("ctc_loss takes float32 logits")
    _chk(logits, labels, label_len, seq_len)
    T, B, C = logits.shape
    Lmax = labels.shape[1] if labels.dim() == 2 else 0
    labels = labels.reshape(B, Lmax)
    if labels.numel() == 0:
        labels = torch.zeros(B, 1, dtype=torch.int32, device=logits.device)
        Lmax = 1
    nb = _lib.lib().ocrk_ctc_workspace_size(T, B, Lmax)
    ws = _ws(nb, logits.device)
    loss = torch.empty(B, dtype=torch.float32, device=logits.device)
    grad = torch.empty_like(logits) if need_grad else None
    if status is None:
        status = torch.empty(B, dtype=torch.int32, device=logits.device)
    call("ocrk_ctc_loss", ptr(logits), ptr(labels), ptr(label_len), ptr(seq_len), T, B, C, Lmax,
         float(grad_scale), ptr(loss), ptr(grad), ptr(status), ptr(status_word(logits.device)), ptr(ws), nb,
         _stream(logits))
    return loss, grad, status


def ctc_greedy_decode(logits, seq_len, merge_repeated=True):
    """Greedy decode. Returns (out i64 [B,T] -1 padded, out_len i32 [B], neg_sum f32 [B])."""
    if logits.dtype != torch.float32:
        raise TypeError("ctc_greedy_decode takes float32 logits")
    _chk(logits, seq_len)
    T, B, C = logits.shape
    out = torch.empty(B, T, dtype=torch.int64, device=logits.device)
    out_len = torch.empty(B, dtype=torch.int32, device=logits.device)
    neg = torch.empty(B, dtype=torch.float32, device=logits.device)
    call("ocrk_ctc_greedy_decode", ptr(logits), ptr(seq_len), T, B, C, int(bool(merge_repeated)),
         ptr(out), ptr(out_len), ptr(neg), _stream(logits))
    return out, out_len, neg


def ctc_beam_decode(logits, seq_len, beam_width=100, top_paths=1, merge_repeated=True):
    """Prefix beam search. Returns (out i64 [top_paths,B,T] -1 padded,
    out_len i32 [top_paths,B], log_probs f32 [B,top_paths])."""
    if logits.dtype != torch.float32:
        raise TypeError("ctc_beam_decode takes float32 logits")
    _chk(logits, seq_len)
    T, B, C = logits.shape
    dev = logits.device
    out = torch.empty(top_paths, B, T, dtype=torch.int64, device=dev)
    out_len = torch.empty(top_paths, B, dtype=torch.int32, device=dev)
    logp = torch.empty(B, top_paths, dtype=torch.float32, device=dev)
    nb = _lib.lib().ocrk_ctc_beam_workspace_size(T, B, int(beam_width))
    ws = _ws(nb, dev)
    call("ocrk_ctc_beam_decode", ptr(logits), ptr(seq_len), T, B, C, int(beam_width), int(top_paths),
         int(bool(merge_repeated)), ptr(out), ptr(out_len), ptr(logp), ptr(ws), nb, _stream(logits))
    return out, out_len, logp


def edit_distance(hyp, hyp_len, labels, label_len, totals=None):
    """Levenshtein distance per row (tf.edit_distance normalize=False).
    hyp i64 [B,S] with hyp_len i32 [B]; labels i32 [B,L] with label_len i32 [B].
    Returns dist f32 [B]; accumulates {sum, nonzero, sum label_len} into
    `totals` (i32 [3]) when given."""
    _chk(hyp, hyp_len, labels, label_len)
    B = hyp.shape[0]
    # a batch whose decodes are all empty (or all-empty labels) has a 0-column
    # tensor, i.e. no storage: give the kernel one padding column (lengths rule)
    if hyp.shape[1] == 0:
        hyp = torch.full((B, 1), -1, dtype=hyp.dtype, device=hyp.device)
    if labels.shape[1] == 0:
        labels = torch.zeros((B, 1), dtype=labels.dtype, device=labels.device)
    dist = torch.empty(B, dtype=torch.float32, device=hyp.device)
    if totals is not None:
        _chk(totals)
    call("ocrk_edit_distance", ptr(hyp), ptr(hyp_len), hyp.shape[1], ptr(labels), ptr(label_len),
         labels.shape[1], B, ptr(dist), ptr(totals) if totals is not None else None, _stream(hyp))
    return dist
