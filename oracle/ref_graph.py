"""NumPy restatement of the reference graph -- TEST INFRASTRUCTURE ONLY.

Each function cites the reference file:line whose behaviour it restates
(paths relative to the reference repo root), and marks TensorFlow-1 op
semantics it relies on with [TF1]. Everything here is plain NumPy so it runs
on any host; dtype defaults to float32 (the reference's dtype) and every
function also works in float64 for known-answer tests.
"""
import numpy as np

# ----------------------------------------------------------------- constants
# src/weinman/mjsynth.py:23
OUT_CHARSET = ("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789 "
               "`~!@#$%^&*()-=_+[]{};'\\:\"|,./<>?")
NUM_CLASSES = len(OUT_CHARSET)          # mjsynth.py:25-26 -> 95
BLANK = NUM_CLASSES                     # [TF1] ctc blank = num_classes - 1 of the 96 logits

# src/weinman/model.py:47-54: (filters, kernel, padding, name, batch_norm)
LAYER_PARAMS = [(32, 3, "valid", "conv1", False),
                (32, 3, "same", "conv2", True),
                (64, 3, "same", "conv3", False),
                (64, 3, "same", "conv4", True),
                (128, 3, "same", "conv5", False),
                (128, 3, "same", "conv6", True),
                (256, 3, "same", "conv7", False),
                (256, 3, "same", "conv8", True)]
# pools after conv2/4/6/8 (model.py:136,139,142,145): (kh, kw, sh, sw)
POOLS = {"conv2": (2, 2, 2, 2), "conv4": (2, 2, 2, 1), "conv6": (2, 2, 2, 1), "conv8": (3, 1, 3, 1)}
BN_EPS = 1e-3                           # [TF1] tf.layers.batch_normalization default
BN_MOMENTUM = 0.99                      # [TF1] idem
FORGET_BIAS = 1.0                       # [TF1] LSTMCell default


class InfeasibleLabelError(ValueError):
    """[TF1] ctc_loss InvalidArgument: 'Not enough time for target transition sequence'."""


# ------------------------------------------------------------ a1 preprocess
def preprocess(img_u8):
    """validate._preprocess_image (src/weinman/validate.py:56-68).

    [TF1] convert_image_dtype(uint8 -> float32) = cast * float32(1/255); then -0.5.
    """
    x = img_u8.astype(np.float32) * np.float32(1.0 / 255.0)
    return x - np.float32(0.5)


def preprocess_train(img_u8):
    """mjsynth._preprocess_image (src/weinman/mjsynth.py:185-194): also duplicates
    the first row (H 31 -> 32). img_u8 is one HWC image."""
    x = preprocess(img_u8)
    return np.concatenate([x[:1], x], axis=0)


def seq_len_from_width(widths):
    """convnet_layers tail (src/weinman/model.py:152-163): floor((w-2)/2) - 2."""
    w = np.asarray(widths, dtype=np.int32)
    return ((w - 2) // 2 - 1 - 1).astype(np.int32)


def encode_text(text):
    """Label indices of a string (mjsynth-tfrecord.py:149-150 uses out_charset.index)."""
    return [OUT_CHARSET.index(ch) for ch in text]


def get_string(labels):
    """validate._get_string (src/weinman/validate.py:126-129)."""
    return "".join(OUT_CHARSET[int(c)] for c in labels)


# ------------------------------------------------------------------- a2 conv
def _windows(x, kh, kw, sh=1, sw=1):
    B, H, W, C = x.shape
    Ho, Wo = (H - kh) // sh + 1, (W - kw) // sw + 1
    s = x.strides
    return np.lib.stride_tricks.as_strided(
        x, (B, Ho, Wo, kh, kw, C), (s[0], s[1] * sh, s[2] * sw, s[1], s[2], s[3]), writeable=False)


def _pad_same(x, k):
    p = k // 2
    return np.pad(x, ((0, 0), (p, p), (p, p), (0, 0)))


def conv2d(x, kernel, bias, padding):
    """tf.layers.conv2d, stride 1, NHWC x, HWIO kernel (src/weinman/model.py:97-104).
    [TF1] 'same' with odd k pads k//2 on each side; 'valid' pads nothing."""
    k = kernel.shape[0]
    xp = _pad_same(x, k) if padding == "same" else x
    cols = np.ascontiguousarray(_windows(xp, k, k))
    y = np.tensordot(cols, kernel, axes=([3, 4, 5], [0, 1, 2]))
    return (y + bias).astype(x.dtype, copy=False)


def conv2d_bwd(x, kernel, dy, padding, need_dx=True):
    """Gradients of conv2d w.r.t. input, kernel and bias."""
    k = kernel.shape[0]
    xp = _pad_same(x, k) if padding == "same" else x
    cols = np.ascontiguousarray(_windows(xp, k, k))
    dw = np.tensordot(cols, dy, axes=([0, 1, 2], [0, 1, 2])).astype(x.dtype, copy=False)
    db = dy.sum(axis=(0, 1, 2))
    dx = None
    if need_dx:
        # full correlation of dy with the flipped, transposed kernel
        p = k - 1 - (k // 2 if padding == "same" else 0)
        dyp = np.pad(dy, ((0, 0), (p, p), (p, p), (0, 0)))
        wf = kernel[::-1, ::-1].transpose(0, 1, 3, 2)
        dcols = np.ascontiguousarray(_windows(dyp, k, k))
        dx = np.tensordot(dcols, wf, axes=([3, 4, 5], [0, 1, 2])).astype(x.dtype, copy=False)
    return dx, dw, db


def relu(x):
    return np.maximum(x, 0)


def relu_bwd(y, dy):
    """[TF1] ReluGrad: dy * (y > 0)."""
    return dy * (y > 0)


# --------------------------------------------------------------- a3 batch norm
def bn_train(x, gamma, beta, eps=BN_EPS):
    """norm_layer in TRAIN mode (src/weinman/model.py:118-123).
    [TF1] fused batch norm: batch mean / biased variance over N,H,W normalise;
    returns (y, mean, biased var, unbiased var for the moving average, cache)."""
    axes = (0, 1, 2)
    n = x.size // x.shape[-1]
    mean = x.mean(axis=axes, dtype=np.float64)
    var = ((x - mean) ** 2).mean(axis=axes, dtype=np.float64)
    inv = 1.0 / np.sqrt(var + eps)
    xhat = ((x - mean) * inv).astype(x.dtype)
    y = (gamma * xhat + beta).astype(x.dtype)
    var_unbiased = var * n / max(n - 1, 1)
    return y, mean.astype(x.dtype), var.astype(x.dtype), var_unbiased.astype(x.dtype), (xhat, inv)


def bn_infer(x, gamma, beta, moving_mean, moving_var, eps=BN_EPS):
    """norm_layer in INFER mode: moving statistics."""
    inv = 1.0 / np.sqrt(moving_var.astype(np.float64) + eps)
    return (gamma * ((x - moving_mean) * inv) + beta).astype(x.dtype)


def bn_bwd(dy, cache, gamma):
    xhat, inv = cache
    axes = (0, 1, 2)
    n = dy.size // dy.shape[-1]
    dbeta = dy.sum(axis=axes, dtype=np.float64)
    dgamma = (dy * xhat).sum(axis=axes, dtype=np.float64)
    dx = (gamma * inv) * (dy - dbeta / n - xhat * (dgamma / n))
    return dx.astype(dy.dtype), dgamma.astype(dy.dtype), dbeta.astype(dy.dtype)


def bn_moving_update(moving, value, momentum=BN_MOMENTUM):
    """[TF1] assign_moving_average: moving -= (moving - value) * (1 - momentum)."""
    return moving - (moving - value) * np.asarray(1.0 - momentum, dtype=moving.dtype)


# ------------------------------------------------------------------ a4 pooling
def maxpool(x, kh, kw, sh, sw):
    """pool_layer / pool8 (src/weinman/model.py:111-116,145-146), 'valid'."""
    return _windows(x, kh, kw, sh, sw).max(axis=(3, 4))


def maxpool_bwd(x, dy, kh, kw, sh, sw):
    """[TF1] MaxPoolGrad: each output's gradient goes to the first maximum of
    its window in row-major scan order; overlapping windows accumulate."""
    B, Ho, Wo, C = dy.shape
    win = _windows(x, kh, kw, sh, sw).reshape(B, Ho, Wo, kh * kw, C)
    idx = win.argmax(axis=3)                       # first max
    hh = np.arange(Ho)[None, :, None, None] * sh + idx // kw
    ww = np.arange(Wo)[None, None, :, None] * sw + idx % kw
    bb = np.broadcast_to(np.arange(B)[:, None, None, None], idx.shape)
    cc = np.broadcast_to(np.arange(C)[None, None, None, :], idx.shape)
    dx = np.zeros_like(x)
    np.add.at(dx, (bb, hh, ww, cc), dy)
    return dx


# --------------------------------------------------------------- a7' LSTM cell
def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_cell(x, h, c, kernel, bias, forget_bias=FORGET_BIAS):
    """[TF1] rnn_cell_impl.LSTMCell.call (no peepholes, no projection):
    [i, j, f, o] = [x, h] @ kernel + bias; c' = sig(f + fb) c + sig(i) tanh(j);
    h' = sig(o) tanh(c'). Used by model_bu.py:173-180."""
    z = np.concatenate([x, h], axis=1) @ kernel + bias
    i, j, f, o = np.split(z, 4, axis=1)
    si, tj, sf, so = _sigmoid(i), np.tanh(j), _sigmoid(f + forget_bias), _sigmoid(o)
    c_new = sf * c + si * tj
    tc = np.tanh(c_new)
    h_new = so * tc
    return h_new, c_new, (si, tj, sf, so, tc)


def gru_cell(x, h, gate_kernel, gate_bias, cand_kernel, cand_bias):
    """[TF1] rnn_cell_impl.GRUCell.call (src/weinman/model.py:173-180):
    [r, u] = sig([x, h] @ Wg + bg); c = tanh([x, r*h] @ Wc + bc);
    h' = u h + (1 - u) c. The reset gate multiplies h BEFORE the matmul."""
    g = _sigmoid(np.concatenate([x, h], axis=1) @ gate_kernel + gate_bias)
    r, u = np.split(g, 2, axis=1)
    cand = np.tanh(np.concatenate([x, r * h], axis=1) @ cand_kernel + cand_bias)
    h_new = u * h + (1 - u) * cand
    return h_new, (r, u, cand)


def _step_index(s, seq_len, reverse):
    """Time index each batch row reads at recurrence step s.
    [TF1] bidirectional_dynamic_rnn: the bw cell runs over
    reverse_sequence(inputs, seq_len) -> step s < len reads x[len-1-s]."""
    if not reverse:
        return np.full(seq_len.shape, s, dtype=np.int64)
    return np.where(s < seq_len, seq_len - 1 - s, s).astype(np.int64)


def lstm_dir_fwd(x, seq_len, kernel, bias, reverse):
    """One direction of dynamic_rnn(time_major, sequence_length):
    [TF1] for steps >= seq_len the output is 0 and the state is carried."""
    T, B, _ = x.shape
    H = kernel.shape[1] // 4
    h = np.zeros((B, H), x.dtype)
    c = np.zeros((B, H), x.dtype)
    out = np.zeros((T, B, H), x.dtype)
    cache = []
    rows = np.arange(B)
    for s in range(T):
        valid = s < seq_len
        t_idx = _step_index(s, seq_len, reverse)
        xs = x[t_idx, rows]
        h_new, c_new, acts = lstm_cell(xs, h, c, kernel, bias)
        cache.append((t_idx, valid, xs, h, c, acts))
        v = valid[:, None]
        out[t_idx[valid], rows[valid]] = h_new[valid]
        h = np.where(v, h_new, h).astype(x.dtype)
        c = np.where(v, c_new, c).astype(x.dtype)
    return out, cache


def lstm_dir_bwd(dout, cache, kernel, n_in):
    """BPTT for lstm_dir_fwd. Returns dx (same layout as x), dkernel, dbias."""
    T, B, H = dout.shape
    dx = np.zeros((T, B, n_in), dout.dtype)
    dk = np.zeros_like(kernel)
    db = np.zeros(kernel.shape[1], dout.dtype)
    dh = np.zeros((B, H), dout.dtype)
    dc = np.zeros((B, H), dout.dtype)
    rows = np.arange(B)
    wx, wh = kernel[:n_in], kernel[n_in:]
    for s in range(T - 1, -1, -1):
        t_idx, valid, xs, h_prev, c_prev, (si, tj, sf, so, tc) = cache[s]
        v = valid[:, None]
        dh_tot = np.where(v, dh + dout[t_idx, rows], 0)
        dc_tot = np.where(v, dc, 0)
        do = dh_tot * tc * so * (1 - so)
        dct = dc_tot + dh_tot * so * (1 - tc * tc)
        di = dct * tj * si * (1 - si)
        dj = dct * si * (1 - tj * tj)
        df = dct * c_prev * sf * (1 - sf)
        dz = np.concatenate([di, dj, df, do], axis=1)
        dk += np.concatenate([xs, h_prev], axis=1).T @ dz
        db += dz.sum(axis=0)
        dxs = dz @ wx.T
        np.add.at(dx, (t_idx[valid], rows[valid]), dxs[valid])
        dh = np.where(v, dz @ wh.T, dh)
        dc = np.where(v, dct * sf, dc)
    return dx, dk, db


def gru_dir_fwd(x, seq_len, gk, gb, ck, cb, reverse):
    T, B, _ = x.shape
    H = ck.shape[1]
    h = np.zeros((B, H), x.dtype)
    out = np.zeros((T, B, H), x.dtype)
    cache = []
    rows = np.arange(B)
    for s in range(T):
        valid = s < seq_len
        t_idx = _step_index(s, seq_len, reverse)
        xs = x[t_idx, rows]
        h_new, acts = gru_cell(xs, h, gk, gb, ck, cb)
        cache.append((t_idx, valid, xs, h, acts))
        out[t_idx[valid], rows[valid]] = h_new[valid]
        h = np.where(valid[:, None], h_new, h).astype(x.dtype)
    return out, cache


def gru_dir_bwd(dout, cache, gk, ck, n_in):
    T, B, H = dout.shape
    dx = np.zeros((T, B, n_in), dout.dtype)
    dgk, dck = np.zeros_like(gk), np.zeros_like(ck)
    dgb, dcb = np.zeros(gk.shape[1], dout.dtype), np.zeros(ck.shape[1], dout.dtype)
    dh = np.zeros((B, H), dout.dtype)
    rows = np.arange(B)
    for s in range(T - 1, -1, -1):
        t_idx, valid, xs, h_prev, (r, u, cand) = cache[s]
        v = valid[:, None]
        dh_tot = np.where(v, dh + dout[t_idx, rows], 0)
        du = dh_tot * (h_prev - cand)
        dcand = dh_tot * (1 - u)
        dzc = dcand * (1 - cand * cand)
        xr = np.concatenate([xs, r * h_prev], axis=1)
        dck += xr.T @ dzc
        dcb += dzc.sum(axis=0)
        dxr = dzc @ ck.T
        dx_c, drh = dxr[:, :n_in], dxr[:, n_in:]
        dr = drh * h_prev
        dzg = np.concatenate([dr * r * (1 - r), du * u * (1 - u)], axis=1)
        xh = np.concatenate([xs, h_prev], axis=1)
        dgk += xh.T @ dzg
        dgb += dzg.sum(axis=0)
        dxh = dzg @ gk.T
        dxs = dx_c + dxh[:, :n_in]
        dh_prev = dh_tot * u + drh * r + dxh[:, n_in:]
        np.add.at(dx, (t_idx[valid], rows[valid]), dxs[valid])
        dh = np.where(v, dh_prev, dh)
    return dx, dgk, dgb, dck, dcb


# ------------------------------------------------------------------- a9 CTC
def log_softmax(x, axis=-1):
    m = x.max(axis=axis, keepdims=True)
    z = x - m
    return z - np.log(np.exp(z).sum(axis=axis, keepdims=True))


def ctc_required_time(labels):
    """[TF1] ctc_loss_calculator: required = L + #(consecutive repeats)."""
    labels = list(labels)
    return len(labels) + sum(1 for a, b in zip(labels, labels[1:]) if a == b)


def ctc_loss_single(logits, labels, blank=BLANK):
    """-log p(labels | logits[:T]) and its gradient w.r.t. the logits.

    [TF1] tf.nn.ctc_loss (model.py:226) with preprocess_collapse_repeated=False,
    ctc_merge_repeated=True, softmax taken inside. alpha includes the emission at
    t, beta excludes it, so grad = softmax - sum_{s: l'_s = k} a_t(s) b_t(s) / p.
    logits: [T, C] for one sequence (already cut to its seq_len).
    """
    T, C = logits.shape
    lab = list(int(v) for v in labels)
    if ctc_required_time(lab) > T:
        raise InfeasibleLabelError(
            f"Not enough time for target transition sequence (required: "
            f"{ctc_required_time(lab)}, available: {T})")
    lp = log_softmax(logits.astype(np.float64))
    lprime = [blank]
    for v in lab:
        lprime += [v, blank]
    S = len(lprime)
    lprime = np.array(lprime)
    skip = np.zeros(S, bool)                       # transition s-2 -> s allowed
    skip[2:] = (lprime[2:] != blank) & (lprime[2:] != lprime[:-2])
    NEG = -np.inf
    la = np.full((T, S), NEG)
    la[0, 0] = lp[0, blank]
    if S > 1:
        la[0, 1] = lp[0, lprime[1]]
    def shift(a, k):                               # out[s] = a[s-k] (k>0) / a[s+|k|]
        out = np.full(S, NEG)
        if k > 0:
            out[k:] = a[:S - k]
        else:
            out[:S + k] = a[-k:]
        return out

    for t in range(1, T):
        a = la[t - 1]
        a1 = shift(a, 1)
        a2 = np.where(skip, shift(a, 2), NEG)
        la[t] = np.logaddexp(np.logaddexp(a, a1), a2) + lp[t, lprime]
    lb = np.full((T, S), NEG)
    lb[T - 1, S - 1] = 0.0
    if S > 1:
        lb[T - 1, S - 2] = 0.0
    skip_next = np.zeros(S, bool)                  # s -> s+2 allowed
    skip_next[:S - 2] = skip[2:]
    for t in range(T - 2, -1, -1):
        nb = lb[t + 1] + lp[t + 1, lprime]
        b1 = shift(nb, -1)
        b2 = np.where(skip_next, shift(nb, -2), NEG)
        lb[t] = np.logaddexp(np.logaddexp(nb, b1), b2)
    logp = np.logaddexp(la[T - 1, S - 1], la[T - 1, S - 2]) if S > 1 else la[T - 1, 0]
    ab = la + lb - logp                            # [T, S] log occupation
    occ = np.zeros((T, C))
    for s in range(S):
        occ[:, lprime[s]] += np.exp(ab[:, s])
    grad = np.exp(lp) - occ
    return -logp, grad


def ctc_loss(logits, labels, seq_len, blank=BLANK):
    """Batched ctc_loss, time-major logits [T, B, C]. Returns per-sequence
    losses [B] and dloss_b/dlogits [T, B, C] (zero for t >= seq_len)."""
    T, B, C = logits.shape
    losses = np.zeros(B)
    grad = np.zeros((T, B, C))
    for b in range(B):
        L = int(seq_len[b])
        loss, g = ctc_loss_single(logits[:L, b], labels[b], blank)
        losses[b] = loss
        grad[:L, b] = g
    return losses, grad


def ctc_loss_bruteforce(logits, labels, blank=BLANK):
    """Known-answer oracle for tiny T, C: enumerate every path, collapse it
    (merge repeats, drop blanks) and sum the probabilities of those that
    produce `labels`. Returns -log p."""
    import itertools
    T, C = logits.shape
    p = np.exp(log_softmax(logits.astype(np.float64)))
    target = tuple(labels)
    total = 0.0
    for path in itertools.product(range(C), repeat=T):
        out, prev = [], None
        for k in path:
            if k != blank and k != prev:
                out.append(k)
            prev = k
        if tuple(out) == target:
            total += np.prod([p[t, k] for t, k in enumerate(path)])
    return -np.log(total)


# ---------------------------------------------------------- a10 greedy decode
def ctc_greedy_decode(logits, seq_len, merge_repeated=True, blank=BLANK):
    """validate._get_output (src/weinman/validate.py:81-92).
    [TF1] CTCGreedyDecoder: per t < seq_len take the first maximum; emit it if
    it is not blank and (not merge_repeated or differs from the previous
    argmax); neg_sum_logits = -sum_t max logit. Returns (list of label lists,
    neg_sum_logits [B])."""
    T, B, C = logits.shape
    seqs = []
    neg = np.zeros(B, dtype=np.float64)
    for b in range(B):
        out, prev = [], -1
        for t in range(int(seq_len[b])):
            k = int(np.argmax(logits[t, b]))
            neg[b] -= float(logits[t, b, k])
            if k != blank and not (merge_repeated and k == prev):
                out.append(k)
            prev = k
        seqs.append(out)
    return seqs, neg


def to_dense(seqs, default=-1):
    """sparse_tensor_to_dense(default_value=-1) (validate.py:91):
    int64 [B, max_len_in_batch]."""
    width = max([len(s) for s in seqs] + [0])
    out = np.full((len(seqs), width), default, dtype=np.int64)
    for i, s in enumerate(seqs):
        out[i, :len(s)] = s
    return out


# ------------------------------------------------------------ a14 edit / CER
def edit_distance(hyp, truth):
    """[TF1] tf.edit_distance(normalize=False) on one pair (test.py:90)."""
    m, n = len(hyp), len(truth)
    d = np.arange(n + 1)
    for i in range(1, m + 1):
        prev, d[0] = d[0], i
        for j in range(1, n + 1):
            cur = d[j]
            d[j] = min(d[j] + 1, d[j - 1] + 1, prev + (hyp[i - 1] != truth[j - 1]))
            prev = cur
    return int(d[n])


def label_and_sequence_error(hyps, truths):
    """test.py:90-99: CER = sum(edit)/sum(len(label)), seq_err = mean(edit>0)."""
    e = [edit_distance(h, t) for h, t in zip(hyps, truths)]
    total = sum(len(t) for t in truths)
    return (sum(e) / total if total else 0.0), float(np.mean([x > 0 for x in e]))


# --------------------------------------------------------------- a13 Adam
def learning_rate(step, base=1e-4, decay_steps=2 ** 16, decay_rate=0.9, staircase=False):
    """train.py:120-126: exponential_decay(1e-4, global_step, 2^16, 0.9)."""
    e = step / decay_steps
    if staircase:
        e = np.floor(e)
    return base * decay_rate ** e


def adam_update(p, g, m, v, lr, t, beta1=0.9, beta2=0.999, eps=1e-8):
    """[TF1] ApplyAdam (train.py:128-137; t = 1-based step):
    lr_t = lr sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
    p -= lr_t m / (sqrt(v) + eps)."""
    lr_t = lr * np.sqrt(1 - beta2 ** t) / (1 - beta1 ** t)
    m = m + (g - m) * (1 - beta1)
    v = v + (g * g - v) * (1 - beta2)
    p = p - lr_t * m / (np.sqrt(v) + eps)
    return p, m, v


# --------------------------------------------------------- a11 beam decode
class _BeamEntry:
    """[TF1] ctc_beam_search.h BeamEntry: prefix-tree node with (total, blank,
    label) log-probabilities at t-1 (oldp) and t (newp)."""
    __slots__ = ("parent", "label", "children", "oldp", "newp")

    def __init__(self, parent, label):
        self.parent, self.label, self.children = parent, label, None
        self.oldp = [-np.inf, -np.inf, -np.inf]     # total, blank, label
        self.newp = [-np.inf, -np.inf, -np.inf]

    def active(self):
        return self.newp[0] != -np.inf

    def label_seq(self, merge_repeated):
        out, prev, e = [], -1, self
        while e.parent is not None:
            if not merge_repeated or e.label != prev:
                out.append(e.label)
            prev = e.label
            e = e.parent
        return out[::-1]


def _lse(a, b):
    """[TF1] ctc_loss_util.h LogSumExp: the smaller added to the larger (in the
    operands' own precision: float64, or float32 as TF computes it)."""
    if a == -np.inf:
        return b
    if b == -np.inf:
        return a
    return a + np.log1p(np.exp(b - a)) if a > b else b + np.log1p(np.exp(a - b))


def ctc_beam_search_single(logits, beam_width, top_paths=1, merge_repeated=True, blank=None, margins=None,
                           dtype=np.float64):
    """One sequence of [TF1] CTCBeamSearchDecoder with the default scorer
    (test.py:84-88 beam 128; client.py:227-231 merge_repeated=False).
    logits [T, C] (already cut to seq_len). Each frame is normalised to
    log-softmax (row max subtracted, then the log-sum-exp), as SURVEY a11
    states for the TF1 decoder's input; leaves are a bounded top-N by
    newp.total with strict '>' against the bottom; ties keep the earlier
    insertion. Returns (paths, log_probs). dtype: the arithmetic -- float64
    (exact-as-possible) or float32 (TF1's own: BeamProbability and LogSumExp
    are float).

    margins: a list that receives every NONZERO decision margin of the search
    (test infrastructure): a branch's oldp.total against the bottom when it is
    gated, an offered child's total against the bottom, and the gaps between
    consecutive leaves at each step's end (their order is the next step's
    processing order). Exact ties (ReLU-zero logits give many) are decided by
    insertion order identically in any precision; a search whose smallest
    nonzero margin is below float32's resolution may legitimately take
    another branch in a float32 implementation (TF's, the GPU kernel's)."""
    T, C = logits.shape
    blank = C - 1 if blank is None else blank
    ninf = dtype(-np.inf)
    root = _BeamEntry(None, -1)
    root.newp = [dtype(0.0), dtype(0.0), ninf]
    leaves = [root]                        # kept sorted by newp.total desc (stable)

    def bottom():
        return leaves[-1]

    def push(e):                           # TopN push: insert keeping descending, stable
        i = len(leaves)
        while i > 0 and leaves[i - 1].newp[0] < e.newp[0]:
            i -= 1
        leaves.insert(i, e)
        if len(leaves) > beam_width:
            leaves.pop()

    for t in range(T):
        x = logits[t].astype(dtype)
        x = x - x.max()
        x = x - np.log(np.exp(x).sum(dtype=dtype))
        branches = list(leaves)            # Extract(): descending newp.total
        leaves = []
        for b in branches:
            b.oldp = list(b.newp)
        for b in branches:
            if b.parent is not None:
                if b.parent.active():
                    prev = b.parent.oldp[1] if b.label == b.parent.label else b.parent.oldp[0]
                    b.newp[2] = _lse(b.newp[2], prev)
                b.newp[2] += x[b.label]
            b.newp[1] = b.oldp[0] + x[blank]
            b.newp[0] = _lse(b.newp[1], b.newp[2])
            push(b)

        def is_candidate(p):
            if margins is not None and p[0] > -np.inf and len(leaves) >= beam_width:
                m = abs(p[0] - bottom().newp[0])
                if m > 0:
                    margins.append(m)
            return p[0] > -np.inf and (len(leaves) < beam_width or p[0] > bottom().newp[0])

        for b in branches:
            if not is_candidate(b.oldp):
                continue
            if b.children is None:
                b.children = [_BeamEntry(b, l) for l in range(C) if l != blank]
            for c in b.children:
                if c.active():
                    continue
                c.newp[1] = ninf
                prev = b.oldp[1] if c.label == b.label else b.oldp[0]
                c.newp[2] = x[c.label] + prev
                c.newp[0] = c.newp[2]
                if is_candidate(c.newp):
                    if len(leaves) == beam_width:
                        bottom().newp = [ninf, ninf, ninf]
                    push(c)
                else:
                    c.oldp = [ninf, ninf, ninf]
                    c.newp = [ninf, ninf, ninf]
        if margins is not None:
            margins += [m for m in (a.newp[0] - b.newp[0] for a, b in zip(leaves, leaves[1:])) if m > 0]
    top = leaves[:top_paths]
    return [e.label_seq(merge_repeated) for e in top], [e.newp[0] for e in top]


def ctc_beam_search_min_margin(logits, seq_len, beam_width, merge_repeated=True, dtype=np.float64):
    """Smallest nonzero decision margin (log-prob units) of the search over one
    sequence (logits [T, 1, C] or [T, C]); +inf when every decision is exact."""
    lg = logits[:, 0] if logits.ndim == 3 else logits
    margins = []
    ctc_beam_search_single(lg[:int(np.asarray(seq_len).reshape(-1)[0])], beam_width, 1, merge_repeated,
                           margins=margins, dtype=dtype)
    return float(min(margins)) if margins else np.inf


def ctc_beam_search_decode(logits, seq_len, beam_width=100, top_paths=1, merge_repeated=True, dtype=np.float64):
    """Batched tf.nn.ctc_beam_search_decoder: per path k a list of B label
    sequences, and log_probabilities [B, top_paths]."""
    T, B, C = logits.shape
    paths = [[None] * B for _ in range(top_paths)]
    logp = np.full((B, top_paths), -np.inf)
    for b in range(B):
        ps, lps = ctc_beam_search_single(logits[:int(seq_len[b]), b], beam_width, top_paths, merge_repeated,
                                         dtype=dtype)
        for k in range(top_paths):
            paths[k][b] = ps[k] if k < len(ps) else []
            logp[b, k] = lps[k] if k < len(lps) else -np.inf
    return paths, logp
