"""Drop-in for src/weinman/model.py: convnet_layers -> rnn_layers -> ctc_loss_layer.

Same names, argument order and meaning as the reference graph builders, run
eagerly on device tensors:

    features, sequence_length = convnet_layers(inputs, widths, mode)   # model.py:126
    logits = rnn_layers(features, sequence_length, num_classes)        # model.py:202
    loss = ctc_loss_layer(logits, sequence_labels, sequence_length)    # model.py:224

Variables live in a ParamStore (the TF graph's variables): pass `store=` or
install a default with `use_store(...)`. Every op is a torch.autograd.Function
whose forward and backward are libocrk HIP kernels; variable gradients are
written straight into the store's flat gradient buffer (the buffer the
all-reduce and the Adam kernel consume), so those Functions return None for
the variable inputs.

Structure of the launches (NHWC activations, compute dtype = store.cfg.dtype):
  conv block k (k = 1..4) = conv_{2k-1} (+ReLU) -> conv_{2k} -> BN -> ReLU -> pool,
  the last block writing features time-major; then per recurrent layer one
  input-projection GEMM + T recurrent steps; then the logits GEMM (+ReLU);
  then the CTC lattice.
"""
import contextlib

import numpy as np
import torch
import torch.distributed as dist

from . import kernels as K
from . import options
from .config import BN_EPS, BN_MOMENTUM, INFER, LAYER_PARAMS, POOLS, TRAIN, ModelConfig, rnn_size  # noqa: F401
from .params import ParamStore

layer_params = LAYER_PARAMS

_DEFAULT = []


@contextlib.contextmanager
def use_store(store):
    """Make `store` the implicit variable scope (TF get_variable analogue)."""
    _DEFAULT.append(store)
    try:
        yield store
    finally:
        _DEFAULT.pop()


def default_store():
    if not _DEFAULT:
        raise RuntimeError("no ParamStore: pass store= or wrap the calls in model.use_store(store)")
    return _DEFAULT[-1]


def _grad_enabled(*ts):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


# ------------------------------------------------------------------ convnet
def _conv_precision(exact):
    """fp32 training's conv tower runs exact f32 MFMA products (store.f32_conv_exact,
    set by the Trainer): the BN backward amplifies the bf16x3 split's ~2^-16 product
    error ~200x into the tower's gradients; everything else keeps the split."""
    return K.f32_exact() if exact else contextlib.nullcontext()


def _conv_wgrad(split, x, dy, dw):
    """dw += the 3x3 conv weight gradient; split (fp32 training, mixed policy): on the
    bf16 engines over the (hi, lo) planes of x and dy -- a leaf gradient, so the
    split's ~2^-16 product error reaches no other gradient."""
    if split:
        for xa, da in K.split_products(x, dy):
            K.conv3x3_bwd_weight(xa, da, dw)
    else:
        K.conv3x3_bwd_weight(x, dy, dw)


class _ConvBlock(torch.autograd.Function):
    """conv_{2k-1} -> conv_{2k} -> BN -> ReLU -> pool (model.py:134-146)."""

    @staticmethod
    def forward(ctx, x, store, k, training, *variables):
        ctx.exact = store.cfg.dtype == torch.float32 and store.f32_conv_exact
        with _conv_precision(ctx.exact):
            return _ConvBlock._forward(ctx, x, store, k, training)

    @staticmethod
    def _forward(ctx, x, store, k, training):
        dt = store.cfg.dtype
        odd, even = f"conv{2 * k - 1}", f"conv{2 * k}"
        P = store.params
        pe = f"convnet/{even}"
        ctx.bn_sync = None
        ctx.relu_bits = None
        # route decisions the backward must follow are taken here, once (an options.override
        # block may end between the forward and the backward)
        ctx.c1_fused = bool(k == 1 and not ctx.exact and options.get("CONV1_FUSED"))
        ctx.pooled_bn = bool(options.get("POOLED_BN"))
        ctx.conv12_bwd = False
        zs = None
        if (k == 1 and training and dt == torch.bfloat16 and not ctx.exact and options.get("CONV1_FUSED")
                and options.get("CONV12_FUSED") and K.conv12_fwd_ok(x, dt)):
            # conv1 -> conv2 in one row walk: conv1's rows produced into conv2's ring (never
            # re-read from HBM) and their ReLU bit mask written for the backward; y1 only when
            # the backward does not recompute it (ocrk_conv12_bwd)
            ctx.conv12_bwd = bool(options.get("CONV12_BWD") and K.conv12_bwd_ok(x, dt))
            w_nk2, _ = store.conv_images(even, dt)
            y_odd, bits, z12, st12 = K.conv12_fwd(x, P["convnet/conv1/kernel"], P["convnet/conv1/bias"], w_nk2,
                                                  P[pe + "/bias"], want_y1=not ctx.conv12_bwd)
            ctx.relu_bits = bits if ctx.conv12_bwd or K.conv2_bwd_data_conv1_wgrad_ok(z12, x) else None
            zs = (z12, st12)
        elif k == 1 and training and dt == torch.bfloat16 and not ctx.exact and options.get("CONV1_FUSED"):
            # the ReLU's bit mask for the fused conv2 backward-data + conv1 weight gradient
            # (it reads 4 B per pixel instead of y1's 64)
            y_odd, bits = K.conv1_fwd(x, P["convnet/conv1/kernel"], P["convnet/conv1/bias"], dt, relu_bits=True)
            ctx.relu_bits = bits if K.conv2_bwd_data_conv1_wgrad_ok(y_odd, x) else None
        elif k == 1:
            y_odd = K.conv1_fwd(x, P["convnet/conv1/kernel"], P["convnet/conv1/bias"], dt)
        else:
            w_nk, _ = store.conv_images(odd, dt)
            if (training and dt == torch.bfloat16 and not ctx.exact and options.get("RELU_BITS")
                    and K.relu_bits_ok(x.shape, x.shape[3], w_nk.shape[0], store.conv_images(even, dt)[0].shape[0],
                                       dt)):
                # conv_{2k-1}'s ReLU as a bit mask for conv_{2k}'s backward-data (1/16 of the bytes)
                y_odd, ctx.relu_bits = K.conv3x3_fwd_relu_bits(x, w_nk, P[f"convnet/{odd}/bias"])
            else:
                y_odd = K.conv3x3_fwd(x, w_nk, P[f"convnet/{odd}/bias"], relu=True)
        B, H, W, _ = (y_odd if zs is None else zs[0]).shape
        M = B * H * W
        w_nk, _ = store.conv_images(even, dt)
        C = w_nk.shape[0]
        if training:
            if zs is not None:                             # conv2 already ran inside conv12_fwd
                z, stats = zs
                trows = W
            elif K.conv3x3_fwd_rowstats_ok(y_odd, C):
                # conv2 on the row-walking kernel: BN partials per output row
                z, stats = K.conv3x3_fwd_rowstats(y_odd, w_nk, P[pe + "/bias"])
                trows = W
            else:
                stats = torch.empty(K.conv_stats_tiles(M), 2, C, dtype=torch.float32, device=x.device)
                z = K.conv3x3_fwd(y_odd, w_nk, P[pe + "/bias"], relu=False, stats=stats)
                trows = 128
            group = _bn_group(store)
            if group is not None:                          # SyncBN: statistics of all ranks' batches
                mean, invstd, count = K.bn_finalize_sync(stats, M, C, BN_EPS, BN_MOMENTUM,
                                                         store.stats[pe + "/batch_norm/moving_mean"],
                                                         store.stats[pe + "/batch_norm/moving_variance"], trows,
                                                         group)
                ctx.bn_sync = (group, count)
            else:
                mean, invstd = K.bn_finalize(stats, M, C, BN_EPS, BN_MOMENTUM,
                                             store.stats[pe + "/batch_norm/moving_mean"],
                                             store.stats[pe + "/batch_norm/moving_variance"], tile_rows=trows)
        else:
            z = K.conv3x3_fwd(y_odd, w_nk, P[pe + "/bias"], relu=False)
            mean, invstd = K.bn_infer_params(store.stats[pe + "/batch_norm/moving_mean"],
                                             store.stats[pe + "/batch_norm/moving_variance"], BN_EPS)
        p = K.bn_relu_pool_fwd(z, mean, invstd, P[pe + "/batch_norm/gamma"], P[pe + "/batch_norm/beta"],
                               POOLS[even], time_major=(k == 4))
        ctx.store, ctx.k = store, k
        ctx.save_for_backward(x, y_odd, z, mean, invstd, p)
        return p

    @staticmethod
    def backward(ctx, dp):
        with _conv_precision(ctx.exact):
            return _ConvBlock._backward(ctx, dp)

    @staticmethod
    def _backward(ctx, dp):
        store, k = ctx.store, ctx.k
        x, y_odd, z, mean, invstd, pooled = ctx.saved_tensors
        dt = store.cfg.dtype
        P, G = store.params, store.grads
        odd, even = f"conv{2 * k - 1}", f"conv{2 * k}"
        pe, po = f"convnet/{even}", f"convnet/{odd}"
        dp = dp.contiguous()
        if dp.dtype != dt:
            dp = K.cast(dp, dt)
        # the bias-gradient reductions (conv bias in front of the BN with the BN's dgamma, and
        # the odd conv's bias from the data-gradient GEMM's tile column sums) stay in the main
        # stream's order: on the side stream or a lane of their own they measured slower
        # (rounds 3-5, profiles/r5_ab_summary.txt)
        dz = K.bn_relu_pool_bwd(z, dp, mean, invstd, P[pe + "/batch_norm/gamma"], P[pe + "/batch_norm/beta"],
                                POOLS[even], dp_time_major=(k == 4),
                                dgamma=G[pe + "/batch_norm/gamma"], dbeta=G[pe + "/batch_norm/beta"],
                                dbias=G[pe + "/bias"],                  # conv bias grad fused
                                sync=ctx.bn_sync,
                                # dgamma / dbeta from the saved pooled output instead of a walk over z
                                pooled=pooled if ctx.bn_sync is None and ctx.pooled_bn else None)
        B, H, W, C = dz.shape
        if k > 1:
            with _conv_side(store, y_odd, dz, *_conv_late_tensors(store)):   # overlaps the data gradient below
                _conv_late_run(store)
                _conv_wgrad(ctx.exact, y_odd, dz, G[pe + "/kernel"])
        _, w_bwd = store.conv_images(even, dt)
        if ctx.conv12_bwd:
            # the step's tail as ONE row walk: conv2's data gradient contracted into conv1's
            # weight gradient, and conv2's weight gradient on y1 recomputed from the image
            # (the forward wrote no y1); the queued conv3 weight gradient on the side stream
            if store.conv_late:
                with _conv_side(store, *_conv_late_tensors(store)):
                    _conv_late_run(store)
            K.conv12_bwd(dz, w_bwd, x, P["convnet/conv1/kernel"], P["convnet/conv1/bias"], G[pe + "/kernel"],
                         G[po + "/kernel"], G[po + "/bias"], relu_bits=ctx.relu_bits)
            store.join()                                   # side-stream weight gradients are in
            return (None, None, None, None) + (None,) * (len(ctx.needs_input_grad) - 4)
        if ctx.c1_fused and K.conv2_bwd_data_conv1_wgrad_ok(dz, x):
            # the step's tail: conv2's weight gradient (y1, dz) on the side stream beside one
            # pass that is conv2's backward-data and conv1's weight gradient (dy1 is
            # contracted as it is produced, never stored: its only consumer is conv1's dW)
            with _conv_side(store, y_odd, dz, *_conv_late_tensors(store)):
                _conv_late_run(store)
                _conv_wgrad(ctx.exact, y_odd, dz, G[pe + "/kernel"])
            bits = ctx.relu_bits
            K.conv2_bwd_data_conv1_wgrad(dz, w_bwd, None if bits is not None else y_odd, x, G[po + "/kernel"],
                                         G[po + "/bias"], relu_bits=bits)
            store.join()                                   # side-stream weight gradients are in
            return (None, None, None, None) + (None,) * (len(ctx.needs_input_grad) - 4)
        # ReLU of conv_{2k-1} fused; its bias gradient from the GEMM's tile column sums (k > 1)
        if k > 1 and ctx.relu_bits is not None:
            dy_odd = K.conv3x3_bwd_data(dz, w_bwd, dbias=G[po + "/bias"], relu_bits=ctx.relu_bits)
        else:
            dy_odd = K.conv3x3_bwd_data(dz, w_bwd, relu_mask=y_odd, dbias=G[po + "/bias"] if k > 1 else None)
        dx = None
        if k == 1:
            # the step's tail: conv1's weight gradient joins the side stream (behind
            # conv3's) while conv2's runs here, so the two streams end together
            # (measured against conv2's on a third stream beside the data gradient
            # and conv1's after it on this one: 6.39 vs 6.37 ms)
            with _conv_side(store, x, dy_odd, *_conv_late_tensors(store)):
                _conv_late_run(store)
                K.conv1_bwd_weight(x, dy_odd, G[po + "/kernel"], G[po + "/bias"])
            _conv_wgrad(ctx.exact, y_odd, dz, G[pe + "/kernel"])
            store.join()                                   # side-stream weight gradients are in
        else:
            if k > 2 and options.get("CONV_SIDE") and options.get("SIDE_STREAM"):
                # the odd conv's weight gradient joins the next side-stream fork (the lower
                # block's even-conv weight gradient): one fork per block instead of two. Not
                # conv3's (k = 2): deferred to conv2's fork it queued in front of conv2's
                # weight gradient at the step's tail
                store.conv_late.append((lambda x=x, d=dy_odd, dw=G[po + "/kernel"], ex=ctx.exact:
                                        _conv_wgrad(ex, x, d, dw), (x, dy_odd)))
            else:
                with _conv_side(store, x, dy_odd):
                    _conv_wgrad(ctx.exact, x, dy_odd, G[po + "/kernel"])
            if ctx.needs_input_grad[0]:
                _, w_bwd_odd = store.conv_images(odd, dt)
                dx = K.conv3x3_bwd_data(dy_odd, w_bwd_odd)
        return (dx, None, None, None) + (None,) * (len(ctx.needs_input_grad) - 4)


def _bn_group(store):
    """The process group of SyncBN (store.bn_group, set by Trainer(sync_bn=True))
    when it spans more than one rank, else None (per-rank statistics)."""
    g = store.bn_group
    if g is None or not (dist.is_available() and dist.is_initialized()):
        return None
    return g if dist.get_world_size(g) > 1 else None


def _block_variables(store, k):
    names = [f"convnet/conv{2 * k - 1}/kernel", f"convnet/conv{2 * k - 1}/bias",
             f"convnet/conv{2 * k}/kernel", f"convnet/conv{2 * k}/bias",
             f"convnet/conv{2 * k}/batch_norm/gamma", f"convnet/conv{2 * k}/batch_norm/beta"]
    return [store.params[n] for n in names]


def convnet_layers(inputs, widths, mode, store=None):
    """convnet_layers (src/weinman/model.py:126-165).

    inputs: [B, 32, W, 1] -- uint8 pixels (validate._preprocess_image is then
    fused into the first conv) or already preprocessed floats in the compute
    dtype. widths: int [B] true image widths. mode: TRAIN or INFER.
    Returns (features [B, T, 256] (a view of time-major storage), seq_len i32 [B])."""
    store = store or default_store()
    training = mode == TRAIN
    x = inputs
    if x.dim() == 4:
        if x.shape[-1] != 1:
            raise ValueError("inputs must be [batch, 32, width, 1]")
        x = x[..., 0]
    x = x.contiguous()
    if x.dtype not in (torch.uint8, store.cfg.dtype):
        x = K.cast(x, store.cfg.dtype)
    track = torch.is_grad_enabled() and training
    h = x
    for k in (1, 2, 3, 4):
        variables = _block_variables(store, k) if track else []
        if track:
            for v in variables:
                v.requires_grad_(True)
        h = _ConvBlock.apply(h, store, k, training, *variables)
    if not isinstance(widths, torch.Tensor):
        widths = torch.as_tensor(np.asarray(widths), dtype=torch.int32)
    widths = widths.to(device=h.device, dtype=torch.int32)
    sequence_length = K.seq_len(widths)
    return h.transpose(0, 1), sequence_length


# ---------------------------------------------------------------- recurrent
_SIDE_STREAMS = {}


def _new_side_stream(dev, lane):
    """A side stream (non-blocking, torch's). (A CU-masked one measured no change
    once the step runs on a stream of its own -- round 6)"""
    return torch.cuda.Stream(device=dev)


class side_work:
    """Run weight-gradient work on a side stream so it overlaps the next
    (latency-bound) recurrent BPTT on the main stream: the side stream first
    waits for everything issued so far on the main stream; the tensors it
    reads are marked for the caching allocator; its completion event joins the
    store's pending list (ParamStore.join, called before the gradients are
    read: the end of backward, zero_grad, the optimizer step)."""

    def __init__(self, store, *tensors, lane="side"):
        self.store, self.tensors, self.lane = store, tensors, lane

    def __enter__(self):
        dev = self.store.device
        if not options.get("SIDE_STREAM"):                          # measurement toggle
            self.side = None
            return self
        side = _SIDE_STREAMS.get((dev, self.lane))
        if side is None:
            side = _SIDE_STREAMS[(dev, self.lane)] = _new_side_stream(dev, self.lane)
        self.side = side
        K.fork(side, torch.cuda.current_stream(dev))
        self.ctx = torch.cuda.stream(side)
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.side is None:
            return False
        done = torch.cuda.Event()
        done.record(self.side)
        self.ctx.__exit__(*exc)
        for t in self.tensors:
            t.record_stream(self.side)
        self.store.pending.append(done)
        return False


def _conv_late_tensors(store):
    return tuple(t for _, ts in store.conv_late for t in ts)


def _conv_late_run(store):
    """Issue the conv weight gradients queued for this side-stream fork (oldest first).
    Each fork records an event on the main stream -- a ~6.4 us gap before the next
    main-stream kernel in the step (profiles/r5e_step_timeline.txt) -- and the side
    stream is busy past the point a queued gradient could have started, so joining
    the next fork costs that gradient no time."""
    late, store.conv_late = store.conv_late, []
    for fn, _ in late:
        fn()


def _conv_side(store, *tensors):
    """Conv weight gradients on the side stream, overlapping the main stream's
    data-gradient GEMMs and BN backward (option CONV_SIDE=0: issue them inline)."""
    if not options.get("CONV_SIDE"):
        return contextlib.nullcontext()
    return side_work(store, *tensors)


class _BiLSTM(torch.autograd.Function):
    """rnn_layer with LSTMCell (src/weinman/model_bu.py:167-199)."""

    @staticmethod
    def forward(ctx, x, seq_len, store, layer, *variables):
        dt = store.cfg.dtype
        T, B, n_in = x.shape
        H = store.cfg.rnn_sizes[layer - 1]
        wxT, _wx, whT, _wh, bias = store.lstm_images(layer, dt)
        gx = K.gemm(x.view(T * B, n_in), wxT, trans_b=True, bias=bias, out_dtype=dt)   # [T*B, 8H]
        out, hprev, cprev, acts = K.lstm_fwd(gx, whT, seq_len, T, B, H, dt, save=any(ctx.needs_input_grad))
        ctx.store, ctx.layer, ctx.H = store, layer, H
        ctx.save_for_backward(x, seq_len, hprev, cprev, acts)
        return out

    @staticmethod
    def backward(ctx, dout):
        store, layer, H = ctx.store, ctx.layer, ctx.H
        x, seq_len, hprev, cprev, acts = ctx.saved_tensors
        dt = store.cfg.dtype
        T, B, n_in = x.shape
        G4 = 4 * H
        dout = dout.contiguous()
        if dout.dtype != dt:
            dout = K.cast(dout, dt)
        _wxT, wx, _whT, wh, _bias = store.lstm_images(layer, dt)
        # [T,B,2,4H]; the bias gradient (both directions) formed in the BPTT loop
        dG = K.lstm_bwd(wh, seq_len, dout, cprev, acts, T, B, H, dbias=store.flat_bias_pair_grad(layer))
        R = T * B
        dx = None
        pre = f"rnn/bdrnn{layer}"
        # (issue orders measured slower and dropped: the lowest layer's data gradient
        # first, 5.08-5.09 vs 5.08 ms; an upper layer's dW_x deferred behind the lower
        # BPTT, 5.17-5.20 -- profiles/r5_ab_summary.txt)
        with side_work(store, x, hprev, dG):               # overlaps the next layer's BPTT
            gf, gb = store.grads[f"{pre}/fw/lstm_cell/kernel"], store.grads[f"{pre}/bw/lstm_cell/kernel"]
            sk = gf.numel()                                                      # [In+H, 4H] f32 each
            # fp32 on the split (not exact mode): the same GEMMs on the bf16 engines over the
            # (hi, lo) planes, hi.hi + hi.lo + lo.hi -- the weight gradients are leaves, so their
            # ~2^-16 product error reaches no other gradient
            if dt == torch.float32 and not K.f32_mode_exact():
                (xh, xl), (hh, hl), (gh, gl) = K.split_bf16(x), K.split_bf16(hprev), K.split_bf16(dG)
                passes = [(xh, hh, gh), (xh, hh, gl), (xl, hl, gh)]          # hi.hi + hi.lo + lo.hi
            else:
                passes = [(x, hprev, dG)]
            if gb.data_ptr() == gf.data_ptr() + 4 * sk:
                # both directions as one batched GEMM each (batch = direction: dG column
                # block d * 4H, h_prev column block d * H, gradient d * (In+H) * 4H):
                # dW_x = x^T . dG_d ; dW_h = h_prev_d^T . dG_d  (split-K over T*B)
                for _xa, ha, ga in passes:
                    K.gemm(ha.view(R, 2 * H), ga.view(R, 2 * G4), trans_a=True, out=gf[n_in:], accumulate=True,
                           M=H, N=G4, K=R, lda=2 * H, ldb=2 * G4, ldc=G4, batch=2, stride_a=H, stride_b=G4,
                           stride_c=sk, splits=_splits(H, G4, R, batch=2, items=_tn_items(layer)))
                for xa, _ha, ga in passes:
                    K.gemm(xa, ga.view(R, 2 * G4), trans_a=True, out=gf, accumulate=True, M=n_in, N=G4, K=R,
                           lda=n_in, ldb=2 * G4, ldc=G4, batch=2, stride_a=0, stride_b=G4, stride_c=sk,
                           splits=_splits(n_in, G4, R, batch=2, items=_tn_items(layer)))
            else:
                for xa, ha, ga in passes:
                    dg = ga.view(R, 2 * G4)
                    for d, gk in enumerate((gf, gb)):
                        dgd = dg[:, d * G4:]                                     # view, ldb = 8H
                        K.gemm(xa, dgd, trans_a=True, out=gk, accumulate=True, M=n_in, N=G4, K=R, lda=n_in,
                               ldb=2 * G4, ldc=G4, splits=_splits(n_in, G4, R, items=_tn_items(layer)))
                        K.gemm(ha.view(R, 2 * H)[:, d * H:], dgd, trans_a=True, out=gk[n_in:], accumulate=True,
                               M=H, N=G4, K=R, lda=2 * H, ldb=2 * G4, ldc=G4,
                               splits=_splits(H, G4, R, items=_tn_items(layer)))
        if ctx.needs_input_grad[0]:
            dx = K.gemm(dG.view(R, 2 * G4), wx, trans_b=True, out_dtype=dt).view(T, B, n_in)
        return (dx,) + (None,) * (len(ctx.needs_input_grad) - 1)


class _BiGRU(torch.autograd.Function):
    """rnn_layer with GRUCell (src/weinman/model.py:167-199)."""

    @staticmethod
    def forward(ctx, x, seq_len, store, layer, *variables):
        dt = store.cfg.dtype
        T, B, n_in = x.shape
        H = store.cfg.rnn_sizes[layer - 1]
        wxT, _wx, whgT, whcT, _whg, _whc, bias = store.gru_images(layer, dt)
        gx = K.gemm(x.view(T * B, n_in), wxT, trans_b=True, bias=bias, out_dtype=dt)   # [T*B, 6H]
        out, hprev, rh, acts = K.gru_fwd(gx, whgT, whcT, seq_len, T, B, H, dt)
        ctx.store, ctx.layer, ctx.H = store, layer, H
        ctx.save_for_backward(x, seq_len, hprev, rh, acts)
        return out

    @staticmethod
    def backward(ctx, dout):
        store, layer, H = ctx.store, ctx.layer, ctx.H
        x, seq_len, hprev, rh, acts = ctx.saved_tensors
        dt = store.cfg.dtype
        T, B, n_in = x.shape
        G2, G3 = 2 * H, 3 * H
        dout = dout.contiguous()
        if dout.dtype != dt:
            dout = K.cast(dout, dt)
        _wxT, wx, _whgT, _whcT, whg, whc, _bias = store.gru_images(layer, dt)
        # [T,B,2,3H]; the [gates | candidate] bias gradients formed in the BPTT loop
        dG = K.gru_bwd(whg, whc, seq_len, dout, hprev, acts, T, B, H, dbias=store.gru_bias_cat_grad(layer))
        pre = f"rnn/bdrnn{layer}"
        R = T * B
        side = side_work(store, x, hprev, rh, dG)
        side.__enter__()
        gf, gb = store.grads[f"{pre}/fw/gru_cell/gates/kernel"], store.grads[f"{pre}/bw/gru_cell/gates/kernel"]
        cf, cb = store.grads[f"{pre}/fw/gru_cell/candidate/kernel"], store.grads[f"{pre}/bw/gru_cell/candidate/kernel"]
        sk = (gb.data_ptr() - gf.data_ptr()) // 4                  # fw -> bw distance (elements)
        batched = sk > 0 and cb.data_ptr() - cf.data_ptr() == 4 * sk
        if batched:
            # both directions as one batched GEMM each (batch = direction: dG column
            # block d * 3H, h_prev / r*h column block d * H, gradients d * sk apart)
            dg = dG.view(R, 2 * G3)
            hp, rhv = hprev.view(R, 2 * H), rh.view(R, 2 * H)
            K.gemm(x, dg, trans_a=True, out=gf, accumulate=True, M=n_in, N=G2, K=R, lda=n_in, ldb=2 * G3,
                   ldc=G2, batch=2, stride_a=0, stride_b=G3, stride_c=sk, splits=_splits(n_in, G2, R, batch=2, items=_tn_items(layer)))
            K.gemm(hp, dg, trans_a=True, out=gf[n_in:], accumulate=True, M=H, N=G2, K=R, lda=2 * H, ldb=2 * G3,
                   ldc=G2, batch=2, stride_a=H, stride_b=G3, stride_c=sk, splits=_splits(H, G2, R, batch=2, items=_tn_items(layer)))
            K.gemm(x, dg[:, G2:], trans_a=True, out=cf, accumulate=True, M=n_in, N=H, K=R, lda=n_in,
                   ldb=2 * G3, ldc=H, batch=2, stride_a=0, stride_b=G3, stride_c=sk,
                   splits=_splits(n_in, H, R, batch=2, items=_tn_items(layer)))
            K.gemm(rhv, dg[:, G2:], trans_a=True, out=cf[n_in:], accumulate=True, M=H, N=H, K=R, lda=2 * H,
                   ldb=2 * G3, ldc=H, batch=2, stride_a=H, stride_b=G3, stride_c=sk, splits=_splits(H, H, R, batch=2, items=_tn_items(layer)))
        for d, dn in enumerate(() if batched else ("fw", "bw")):
            gk = store.grads[f"{pre}/{dn}/gru_cell/gates/kernel"]               # [In+H, 2H]
            ck = store.grads[f"{pre}/{dn}/gru_cell/candidate/kernel"]           # [In+H, H]
            dgg = dG.view(R, 2 * G3)[:, d * G3:]                                 # (dz_r, dz_u), ld 6H
            dgc = dG.view(R, 2 * G3)[:, d * G3 + G2:]                            # dz_c, ld 6H
            hp = hprev.view(R, 2 * H)[:, d * H:]
            rhd = rh.view(R, 2 * H)[:, d * H:]
            K.gemm(x, dgg, trans_a=True, out=gk, accumulate=True, M=n_in, N=G2, K=R, lda=n_in,
                   ldb=2 * G3, ldc=G2, splits=_splits(n_in, G2, R, items=_tn_items(layer)))
            K.gemm(hp, dgg, trans_a=True, out=gk[n_in:], accumulate=True, M=H, N=G2, K=R, lda=2 * H,
                   ldb=2 * G3, ldc=G2, splits=_splits(H, G2, R, items=_tn_items(layer)))
            K.gemm(x, dgc, trans_a=True, out=ck, accumulate=True, M=n_in, N=H, K=R, lda=n_in,
                   ldb=2 * G3, ldc=H, splits=_splits(n_in, H, R, items=_tn_items(layer)))
            K.gemm(rhd, dgc, trans_a=True, out=ck[n_in:], accumulate=True, M=H, N=H, K=R, lda=2 * H,
                   ldb=2 * G3, ldc=H, splits=_splits(H, H, R, items=_tn_items(layer)))
        side.__exit__(None, None, None)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = K.gemm(dG.view(R, 2 * G3), wx, trans_b=True, out_dtype=dt).view(T, B, n_in)
        return (dx,) + (None,) * (len(ctx.needs_input_grad) - 1)


# the lowest layer's weight gradients run beside the conv backward's main-stream
# kernels (BN backward: 175-212 VGPRs), which cannot share a CU with a 256 x 256
# TN item (2 waves x 216 VGPRs per SIMD): a cap leaves them CUs. Same-box
# A/B (with the conv weight gradients at 192 too, csrc/conv.hip): 5.215-5.228 vs
# 5.286-5.288 ms per step at 192; 160: 5.215-5.225, 176: 5.26, 224: 5.25. With the
# 16-row BPTT and the channel-block conv weight gradients (round 4, 7 same-box
# pairs): 160 5.062-5.091 vs 192 5.081-5.099 ms, 128 5.069-5.094, 224 5.098-5.111


# an upper layer's dW_x is queued behind the lower BPTT and meets the lower layer's
# data gradient when that BPTT ends (a cap of its own measured slower: 192: 5.28,
# 128: 5.34 vs 5.27-5.30 ms at 256)
# (options TN_ITEMS_L1 = 160, TN_ITEMS = 256)
def _tn_items(layer):
    if layer == 1:
        return options.get("TN_ITEMS_L1")
    return options.get("TN_ITEMS")


def _splits(M, N, Kdim, batch=1, items=None):
    """K slices for a weight-gradient GEMM (f32 partials + a fixed-order
    reduce): enough items for the chip. M, N >= 256 run on the 256 x 256
    ping-pong TN engine (one item per CU, slices of >= 1024 rows), smaller
    outputs on the 128 x 128 engine (~2 items per CU, >= 2048 rows). `batch`
    problems share the chip. The 256 x 256 launches stop at OCRK_TN_ITEMS
    (256) items, one round on the chip (round 2 measured 224 faster, 6.23 vs
    6.29 ms; since the TN engines keep their DMAs in flight (round 3) 256 is:
    5.374-5.402 vs 5.416-5.426 ms, 320 / 384 / 512 5.45 / 5.44-5.48 / 5.56-5.58)."""
    if M >= 256 and N >= 256:
        tiles = -(-M // 256) * -(-N // 256) * batch
        return int(max(1, min((items or options.get("TN_ITEMS")) // tiles, Kdim // 1024)))      # <= 256 items: one round on the chip
    tiles = -(-M // 128) * -(-N // 128) * batch
    return int(max(1, min(-(-512 // tiles), Kdim // 2048)))


class _Logits(torch.autograd.Function):
    """tf.layers.dense(num_classes + 1, activation=relu) (model.py:216-220)."""

    @staticmethod
    def forward(ctx, x, store, *variables):
        dt = store.cfg.dtype
        T, B, D = x.shape
        wT = store.logits_image_t(dt)                                   # [C][D]: the NT engine's operand
        logits = K.gemm(x.view(T * B, D), wT, trans_b=True, bias=store.params["rnn/logits/bias"], relu=True)
        logits = logits.view(T, B, -1)
        ctx.store = store
        ctx.save_for_backward(x, logits)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        store = ctx.store
        x, logits = ctx.saved_tensors
        dt = store.cfg.dtype
        T, B, D = x.shape
        C = logits.shape[-1]
        R = T * B
        dpre = K.relu_mask(dlogits.contiguous(), logits, dt)                       # [T,B,C]
        with side_work(store, x, dpre):
            # fp32 on the split: the leaf gradient on the bf16 engines (as the recurrent dW)
            split = dt == torch.float32 and not K.f32_mode_exact() and x.numel() % 8 == 0 and dpre.numel() % 8 == 0
            for xa, pa in (K.split_products(x, dpre) if split else [(x, dpre)]):
                K.gemm(xa, pa, trans_a=True, out=store.grads["rnn/logits/kernel"], accumulate=True,
                       M=D, N=C, K=R, lda=D, ldb=C, ldc=C, splits=_splits(D, C, R))
            K.colsum(dpre, R, C, store.grads["rnn/logits/bias"])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = K.gemm(dpre.view(R, C), store.logits_image(dt), trans_b=True, out_dtype=dt).view(T, B, D)
        return (dx,) + (None,) * (len(ctx.needs_input_grad) - 1)


def rnn_layers(features, sequence_length, num_classes, store=None):
    """rnn_layers (src/weinman/model.py:202-221): time-major transpose, two
    bidirectional recurrent layers, dense + ReLU logits [T, B, num_classes+1]."""
    store = store or default_store()
    cfg = store.cfg
    if num_classes != cfg.num_classes:
        raise ValueError(f"store was built for {cfg.num_classes} classes, got {num_classes}")
    x = features.transpose(0, 1)                                                  # model.py:212
    if not x.is_contiguous():
        x = x.contiguous()
    if x.dtype != cfg.dtype:
        x = K.cast(x, cfg.dtype)
    sequence_length = sequence_length.to(device=x.device, dtype=torch.int32).contiguous()
    # the recurrent step kernels tile the batch by 64 (bf16) / 32 (fp32) rows:
    # pad with zero-length sequences (zero outputs, zero gradients), slice after
    B = x.shape[1]
    mult = 64 if cfg.dtype == torch.bfloat16 else 32
    Bp = -(-B // mult) * mult
    if Bp != B:
        x = torch.cat([x, x.new_zeros(x.shape[0], Bp - B, x.shape[2])], dim=1)
        sequence_length = torch.cat([sequence_length, sequence_length.new_zeros(Bp - B)])
    track = torch.is_grad_enabled() and x.requires_grad
    for layer in range(1, len(cfg.rnn_sizes) + 1):
        variables = []
        if track:
            pre = f"rnn/bdrnn{layer}"
            leaves = ("lstm_cell/kernel", "lstm_cell/bias") if cfg.cell == "lstm" else \
                ("gru_cell/gates/kernel", "gru_cell/gates/bias", "gru_cell/candidate/kernel", "gru_cell/candidate/bias")
            variables = [store.params[f"{pre}/{d}/{v}"] for d in ("fw", "bw") for v in leaves]
        op = _BiLSTM if cfg.cell == "lstm" else _BiGRU
        x = op.apply(x, sequence_length, store, layer, *variables)
    variables = [store.params["rnn/logits/kernel"], store.params["rnn/logits/bias"]] if track else []
    logits = _Logits.apply(x, store, *variables)
    return logits if Bp == B else logits[:, :B]


# ---------------------------------------------------------------------- CTC
class _CTCLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, label_len, seq_len):
        B = logits.shape[1]
        loss_b, grad, status = K.ctc_loss(logits.contiguous(), labels, label_len, seq_len,
                                          grad_scale=1.0 / max(B, 1), need_grad=logits.requires_grad)
        ctx.save_for_backward(grad if grad is not None else loss_b)
        ctx.status = status
        return K.mean(loss_b)                                                      # model.py:228

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        if _UNIT_ARMED[0] and g.data_ptr() in _UNIT_SEEDS and g.dtype == torch.float32:
            return grad, None, None, None          # d loss / d loss = 1 (Trainer's resident seed): x 1 is exact
        return K.mul_scalar_(grad, g.to(torch.float32).contiguous()), None, None, None


# resident scalar 1.0 tensors (one per device, held here for the process so their
# addresses stay theirs) that the Trainer seeds loss.backward with; private, and
# trusted by _CTCLoss.backward only while unit_backward() is armed
_UNIT_SEEDS = {}
_UNIT_BY_DEVICE = {}
_UNIT_ARMED = [False]


def _unit_seed(device):
    t = _UNIT_BY_DEVICE.get(device)
    if t is None:
        t = _UNIT_BY_DEVICE[device] = torch.ones((), dtype=torch.float32, device=device)
        _UNIT_SEEDS[t.data_ptr()] = t
    return t


def unit_backward(loss):
    """loss.backward() seeded from the device's resident f32 1.0: no fill launch,
    and the CTC backward skips its x 1 pass over the logits gradient. The skip is
    armed only for this call (backward is synchronous), and only for that tensor."""
    seed = _unit_seed(loss.device)
    if _UNIT_CHECK and seed.item() != 1.0:
        raise RuntimeError("the resident backward seed was overwritten")
    _UNIT_ARMED[0] = True
    try:
        loss.backward(seed)
    finally:
        _UNIT_ARMED[0] = False


_UNIT_CHECK = False          # tests: verify the seed (a device sync) before every use


def dense_labels(sequence_labels, batch, device):
    """SparseTensor-like labels -> (dense int32 [B, Lmax], lengths int32 [B]).

    Accepts a list of label sequences, a (indices [N,2], values [N], dense_shape)
    triple as produced by the reference input pipeline (mjsynth.py:71-72), or an
    already dense (labels [B, Lmax], label_len [B]) pair of tensors."""
    if isinstance(sequence_labels, (tuple, list)) and len(sequence_labels) == 2 and \
            isinstance(sequence_labels[0], torch.Tensor):
        lab, ln = sequence_labels
        return lab.to(device=device, dtype=torch.int32).contiguous(), ln.to(device=device, dtype=torch.int32)
    if isinstance(sequence_labels, (tuple, list)) and len(sequence_labels) == 3 and \
            np.asarray(sequence_labels[0]).ndim == 2:
        idx, vals, shape = (np.asarray(a) for a in sequence_labels)
        seqs = [[] for _ in range(int(shape[0]))]
        for (b, _t), v in sorted(zip(map(tuple, idx), vals)):
            seqs[int(b)].append(int(v))
    else:
        seqs = [list(map(int, s)) for s in sequence_labels]
    if len(seqs) != batch:
        raise ValueError(f"{len(seqs)} label sequences for a batch of {batch}")
    lmax = max([len(s) for s in seqs] + [1])
    dense = np.zeros((batch, lmax), np.int32)
    for i, s in enumerate(seqs):
        dense[i, :len(s)] = s
    lens = np.array([len(s) for s in seqs], np.int32)
    return torch.from_numpy(dense).to(device), torch.from_numpy(lens).to(device)


def check_feasible(sequence_labels_dense, label_len, seq_len):
    """[TF1] InvalidArgumentError when a label needs more frames than its
    sequence has (L + repeats > seq_len). Host check (one small D2H copy)."""
    lab = sequence_labels_dense.cpu().numpy()
    ln = label_len.cpu().numpy()
    sl = seq_len.cpu().numpy()
    for b in range(lab.shape[0]):
        l = lab[b, :ln[b]]
        need = len(l) + int(np.sum(l[1:] == l[:-1]))
        if need > sl[b]:
            from ._lib import InvalidArgumentError
            raise InvalidArgumentError(3, f"Not enough time for target transition sequence "
                                          f"(required: {need}, available: {sl[b]}), batch {b}")


def host_labels(sequence_labels):
    """True when the labels are host data (a list of sequences or a
    SparseTensor-like triple), i.e. checkable without touching the device."""
    return not (isinstance(sequence_labels, (tuple, list)) and len(sequence_labels) == 2 and
                isinstance(sequence_labels[0], torch.Tensor))


def check_feasible_host(sequence_labels, widths):
    """[TF1] the InvalidArgumentError of tf.nn.ctc_loss (model.py:226,
    ignore_longer_outputs_than_inputs=False) decided on the host, before any
    launch: label + repeats must fit seq_len = floor((w-2)/2) - 2 (model.py:152-163),
    labels must lie in [0, num_classes)."""
    from ._lib import InvalidArgumentError
    from .mjsynth import num_classes
    w = np.asarray(widths.cpu() if isinstance(widths, torch.Tensor) else widths, np.int64).reshape(-1)
    seq = np.floor((w - 2) / 2).astype(np.int64) - 2
    lab, ln = dense_labels(sequence_labels, len(w), "cpu")
    lab, ln = lab.numpy(), ln.numpy()
    for b in range(len(w)):
        row = lab[b, :ln[b]]
        if row.size and (row.min() < 0 or row.max() >= num_classes()):
            raise InvalidArgumentError(3, f"Label values must be in [0, {num_classes()}), batch {b}")
        need = len(row) + int(np.sum(row[1:] == row[:-1]))
        if need > seq[b] or seq[b] <= 0:
            raise InvalidArgumentError(3, f"Not enough time for target transition sequence "
                                          f"(required: {need}, available: {max(int(seq[b]), 0)}), batch {b}")


def ctc_loss_layer(rnn_logits, sequence_labels, sequence_length, check="deferred"):
    """ctc_loss_layer (src/weinman/model.py:224-229): mean over the batch of
    tf.nn.ctc_loss(labels, logits, seq_len, time_major=True).

    A sequence that cannot be scored (label + repeats > seq_len, a bad label
    length or value) gets loss +inf and zero gradient, and the kernel sets a
    bit in the device status word (kernels.status_word). check="deferred"
    (default): the error is raised at the caller's next status check
    (Trainer.step polls the word one step later without a sync, and
    Trainer.check_status / kernels.check_status sync and raise) -- TF raises
    InvalidArgumentError at sess.run; check=True: synchronise now and raise;
    check=False: leave the word to the caller."""
    T, B, _ = rnn_logits.shape
    lab, ln = dense_labels(sequence_labels, B, rnn_logits.device)
    loss = _CTCLoss.apply(rnn_logits, lab, ln, sequence_length.to(torch.int32).contiguous())
    if check is True:
        K.check_status(rnn_logits.device)
    return loss


__all__ = ["convnet_layers", "rnn_layers", "ctc_loss_layer", "layer_params", "rnn_size", "TRAIN", "INFER",
           "ParamStore", "ModelConfig", "use_store", "default_store", "dense_labels", "check_feasible",
           "check_feasible_host", "host_labels"]
