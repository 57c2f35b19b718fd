"""Whole-graph oracle: parameters, forward, backward and one train step --
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates src/weinman/model.py (GRU) / model_bu.py (LSTM, the north-star
BiLSTM) convnet_layers -> rnn_layers -> ctc_loss_layer, and train.py's
Adam step, on NumPy arrays. Parameter names follow the TF1 variable names so
the same dict layout is used by the device implementation.
"""
import numpy as np

from . import ref_graph as G


def param_shapes(cell="lstm", rnn_sizes=(512, 512), num_classes=G.NUM_CLASSES):
    """Trainable variables + BN moving statistics, TF1 names, in creation order."""
    shapes = {}
    cin = 1
    for filters, k, _pad, name, bn in G.LAYER_PARAMS:
        shapes[f"convnet/{name}/kernel"] = (k, k, cin, filters)
        shapes[f"convnet/{name}/bias"] = (filters,)
        if bn:
            for v in ("gamma", "beta", "moving_mean", "moving_variance"):
                shapes[f"convnet/{name}/batch_norm/{v}"] = (filters,)
        cin = filters
    n_in = cin
    for li, H in enumerate(rnn_sizes, start=1):
        for d in ("fw", "bw"):
            pre = f"rnn/bdrnn{li}/{d}"
            if cell == "lstm":
                shapes[f"{pre}/lstm_cell/kernel"] = (n_in + H, 4 * H)
                shapes[f"{pre}/lstm_cell/bias"] = (4 * H,)
            else:
                shapes[f"{pre}/gru_cell/gates/kernel"] = (n_in + H, 2 * H)
                shapes[f"{pre}/gru_cell/gates/bias"] = (2 * H,)
                shapes[f"{pre}/gru_cell/candidate/kernel"] = (n_in + H, H)
                shapes[f"{pre}/gru_cell/candidate/bias"] = (H,)
        n_in = 2 * H
    shapes["rnn/logits/kernel"] = (n_in, num_classes + 1)
    shapes["rnn/logits/bias"] = (num_classes + 1,)
    return shapes


def is_trainable(name):
    return not (name.endswith("moving_mean") or name.endswith("moving_variance"))


def _trunc_normal(rng, shape, std):
    """[TF1] truncated_normal: resample draws beyond 2 std."""
    x = rng.standard_normal(shape)
    bad = np.abs(x) > 2
    while bad.any():
        x[bad] = rng.standard_normal(bad.sum())
        bad = np.abs(x) > 2
    return x * std


def init_params(seed=0, cell="lstm", rnn_sizes=(512, 512), dtype=np.float32):
    """Reference initialisers:
    conv/logits kernels: [TF1] contrib variance_scaling_initializer() =
      truncated normal, std = sqrt(1.3 * 2 / fan_in) (model.py:94, :207);
    biases 0 (model.py:95, :208); BN gamma 1, beta 0, moving mean 0, var 1;
    LSTM kernel trunc-normal std 0.01, bias 0 (model_bu.py:170-180);
    GRU kernels and biases trunc-normal std 0.01 (model.py:170-180)."""
    rng = np.random.default_rng(seed)
    params = {}
    for name, shape in param_shapes(cell, rnn_sizes).items():
        leaf = name.rsplit("/", 1)[1]
        if name.startswith("convnet") and leaf == "kernel":
            fan_in = shape[0] * shape[1] * shape[2]
            val = _trunc_normal(rng, shape, np.sqrt(1.3 * 2.0 / fan_in))
        elif name == "rnn/logits/kernel":
            val = _trunc_normal(rng, shape, np.sqrt(1.3 * 2.0 / shape[0]))
        elif "gru_cell" in name:
            val = _trunc_normal(rng, shape, 0.01)
        elif "lstm_cell" in name and leaf == "kernel":
            val = _trunc_normal(rng, shape, 0.01)
        elif leaf in ("gamma", "moving_variance"):
            val = np.ones(shape)
        else:
            val = np.zeros(shape)
        params[name] = val.astype(dtype)
    return params


class RefModel:
    """Forward/backward of the whole reference graph on one batch."""

    def __init__(self, params, cell="lstm", rnn_sizes=(512, 512)):
        self.p = params
        self.cell = cell
        self.rnn_sizes = tuple(rnn_sizes)

    # ------------------------------------------------------------ convnet
    def convnet_forward(self, x, widths, training):
        """convnet_layers (src/weinman/model.py:126-165). x: float NHWC [B,32,W,1]
        (already preprocessed). Returns features [B,T,256], seq_len [B]."""
        p = self.p
        cache = []
        h = x
        for filters, k, pad, name, bn in G.LAYER_PARAMS:
            pre = f"convnet/{name}"
            z = G.conv2d(h, p[pre + "/kernel"], p[pre + "/bias"], pad)
            ent = {"name": name, "x": h, "pad": pad, "bn": bn}
            if bn:
                g, b = p[pre + "/batch_norm/gamma"], p[pre + "/batch_norm/beta"]
                if training:
                    a, mean, _var, var_u, bcache = G.bn_train(z, g, b)
                    ent["bn_cache"] = bcache
                    ent["batch_mean"], ent["batch_var_unbiased"] = mean, var_u
                else:
                    a = G.bn_infer(z, g, b, p[pre + "/batch_norm/moving_mean"],
                                   p[pre + "/batch_norm/moving_variance"])
                y = G.relu(a)
                kh, kw, sh, sw = G.POOLS[name]
                ent["y"] = y
                ent["pool"] = (kh, kw, sh, sw)
                h = G.maxpool(y, kh, kw, sh, sw)
            else:
                y = G.relu(z)
                ent["y"] = y
                h = y
            cache.append(ent)
        features = h[:, 0]                               # squeeze H (model.py:147)
        self._conv_cache = cache
        return features, G.seq_len_from_width(widths)

    def convnet_backward(self, dfeatures):
        p = self.p
        grads = {}
        dh = dfeatures[:, None]
        for ent in reversed(self._conv_cache):
            name = ent["name"]
            pre = f"convnet/{name}"
            if ent["bn"]:
                kh, kw, sh, sw = ent["pool"]
                dy = G.maxpool_bwd(ent["y"], dh, kh, kw, sh, sw)
                da = G.relu_bwd(ent["y"], dy)
                dz, dgamma, dbeta = G.bn_bwd(da, ent["bn_cache"], p[pre + "/batch_norm/gamma"])
                grads[pre + "/batch_norm/gamma"] = dgamma
                grads[pre + "/batch_norm/beta"] = dbeta
            else:
                dz = G.relu_bwd(ent["y"], dh)
            dx, dw, db = G.conv2d_bwd(ent["x"], p[pre + "/kernel"], dz, ent["pad"],
                                      need_dx=(name != "conv1"))
            grads[pre + "/kernel"] = dw
            grads[pre + "/bias"] = db
            dh = dx
        return grads

    # ---------------------------------------------------------------- rnn
    def rnn_forward(self, features, seq_len):
        """rnn_layers (src/weinman/model.py:202-221). Returns logits [T,B,96]."""
        p = self.p
        x = np.ascontiguousarray(features.transpose(1, 0, 2))   # time-major (:212)
        self._rnn_cache = []
        for li, H in enumerate(self.rnn_sizes, start=1):
            outs, caches = [], []
            for d, rev in (("fw", False), ("bw", True)):
                pre = f"rnn/bdrnn{li}/{d}"
                if self.cell == "lstm":
                    o, c = G.lstm_dir_fwd(x, seq_len, p[pre + "/lstm_cell/kernel"],
                                          p[pre + "/lstm_cell/bias"], rev)
                else:
                    o, c = G.gru_dir_fwd(x, seq_len, p[pre + "/gru_cell/gates/kernel"],
                                         p[pre + "/gru_cell/gates/bias"],
                                         p[pre + "/gru_cell/candidate/kernel"],
                                         p[pre + "/gru_cell/candidate/bias"], rev)
                outs.append(o)
                caches.append(c)
            self._rnn_cache.append((x, caches))
            x = np.concatenate(outs, axis=2)                     # (:197)
        pre_logits = x @ p["rnn/logits/kernel"] + p["rnn/logits/bias"]
        logits = G.relu(pre_logits)                              # (:216-220)
        self._logit_cache = (x, logits)
        return logits

    def rnn_backward(self, dlogits):
        p = self.p
        grads = {}
        x, logits = self._logit_cache
        dpre = G.relu_bwd(logits, dlogits)
        T, B, D = x.shape
        grads["rnn/logits/kernel"] = x.reshape(-1, D).T @ dpre.reshape(T * B, -1)
        grads["rnn/logits/bias"] = dpre.sum(axis=(0, 1))
        dx = dpre @ p["rnn/logits/kernel"].T
        for li in range(len(self.rnn_sizes), 0, -1):
            xin, caches = self._rnn_cache[li - 1]
            H = self.rnn_sizes[li - 1]
            n_in = xin.shape[2]
            dxin = np.zeros_like(xin)
            for di, d in enumerate(("fw", "bw")):
                pre = f"rnn/bdrnn{li}/{d}"
                dout = np.ascontiguousarray(dx[:, :, di * H:(di + 1) * H])
                if self.cell == "lstm":
                    ddx, dk, db = G.lstm_dir_bwd(dout, caches[di], p[pre + "/lstm_cell/kernel"], n_in)
                    grads[pre + "/lstm_cell/kernel"] = dk
                    grads[pre + "/lstm_cell/bias"] = db
                else:
                    ddx, dgk, dgb, dck, dcb = G.gru_dir_bwd(
                        dout, caches[di], p[pre + "/gru_cell/gates/kernel"],
                        p[pre + "/gru_cell/candidate/kernel"], n_in)
                    grads[pre + "/gru_cell/gates/kernel"] = dgk
                    grads[pre + "/gru_cell/gates/bias"] = dgb
                    grads[pre + "/gru_cell/candidate/kernel"] = dck
                    grads[pre + "/gru_cell/candidate/bias"] = dcb
                dxin += ddx
            dx = dxin
        return grads, np.ascontiguousarray(dx.transpose(1, 0, 2))

    # --------------------------------------------------------------- whole
    def forward(self, x, widths, training):
        features, seq_len = self.convnet_forward(x, widths, training)
        return self.rnn_forward(features, seq_len), seq_len

    def loss_and_grads(self, x, widths, labels):
        """ctc_loss_layer (model.py:224-229) in TRAIN mode + full backward.
        Returns (mean loss, grads dict, per-sequence losses, logits, seq_len)."""
        logits, seq_len = self.forward(x, widths, training=True)
        losses, dlog = G.ctc_loss(logits, labels, seq_len)
        B = logits.shape[1]
        dlog = (dlog / B).astype(logits.dtype)                   # reduce_mean
        grads, dfeat = self.rnn_backward(dlog)
        grads.update(self.convnet_backward(dfeat))
        return float(losses.mean()), grads, losses, logits, seq_len

    def bn_moving_updates(self):
        """UPDATE_OPS of the last training forward (train.py:116-118)."""
        new = {}
        for ent in self._conv_cache:
            if ent["bn"]:
                pre = f"convnet/{ent['name']}/batch_norm"
                new[pre + "/moving_mean"] = G.bn_moving_update(self.p[pre + "/moving_mean"], ent["batch_mean"])
                new[pre + "/moving_variance"] = G.bn_moving_update(
                    self.p[pre + "/moving_variance"], ent["batch_var_unbiased"])
        return new


def train_step(params, opt_state, step, x, widths, labels, cell="lstm", rnn_sizes=(512, 512)):
    """One iteration of train.py:196-199: loss, grads, BN moving-average
    updates and an Adam update of every trainable variable. `step` is the
    global_step before the update (0-based). Returns (loss, new params,
    new opt_state)."""
    model = RefModel(params, cell, rnn_sizes)
    loss, grads, _, _, _ = model.loss_and_grads(x, widths, labels)
    lr = G.learning_rate(step)
    new_p = dict(params)
    new_state = {}
    for name, g in grads.items():
        m, v = opt_state.get(name, (np.zeros_like(g), np.zeros_like(g)))
        new_p[name], m, v = G.adam_update(params[name], g, m, v, lr, step + 1)
        new_p[name] = new_p[name].astype(params[name].dtype)
        new_state[name] = (m, v)
    new_p.update(model.bn_moving_updates())
    return loss, new_p, new_state
