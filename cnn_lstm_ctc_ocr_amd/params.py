"""Parameter store: every variable of the reference graph in ONE flat fp32
buffer in HBM (plus a flat gradient buffer and a flat buffer of BatchNorm
moving statistics), addressed by the TF1 variable names of
src/weinman/model.py / model_bu.py (`convnet/conv3/kernel`,
`rnn/bdrnn1/fw/lstm_cell/kernel`, `rnn/logits/bias`, ...).

One buffer means one all-reduce and one Adam launch per step; the per-name
tensors are views. The compute-dtype weight images the kernels read (GEMM
layouts, bf16 casts) are derived from the master copy once per parameter
version (see `images()`).
"""

import numpy as np
import torch

from . import kernels as K
from .config import LAYER_PARAMS, ModelConfig

_ALIGN = 64  # elements (256 B): every view starts 16-B aligned for vector loads


def param_shapes(cfg):
    """(name, shape, trainable) in buffer order. Forward and backward
    direction biases of one recurrent layer sit next to each other so one
    column-sum kernel writes both."""
    out = []
    cin = 1
    for filters, k, _pad, name, bn in LAYER_PARAMS:
        out.append((f"convnet/{name}/kernel", (k, k, cin, filters), True))
        out.append((f"convnet/{name}/bias", (filters,), True))
        if bn:
            out.append((f"convnet/{name}/batch_norm/gamma", (filters,), True))
            out.append((f"convnet/{name}/batch_norm/beta", (filters,), True))
            out.append((f"convnet/{name}/batch_norm/moving_mean", (filters,), False))
            out.append((f"convnet/{name}/batch_norm/moving_variance", (filters,), False))
        cin = filters
    n_in = cin
    for li, H in enumerate(cfg.rnn_sizes, start=1):
        pre = f"rnn/bdrnn{li}"
        if cfg.cell == "lstm":
            for d in ("fw", "bw"):
                out.append((f"{pre}/{d}/lstm_cell/kernel", (n_in + H, 4 * H), True))
            for d in ("fw", "bw"):
                out.append((f"{pre}/{d}/lstm_cell/bias", (4 * H,), True))
        else:
            for d in ("fw", "bw"):
                out.append((f"{pre}/{d}/gru_cell/gates/kernel", (n_in + H, 2 * H), True))
                out.append((f"{pre}/{d}/gru_cell/candidate/kernel", (n_in + H, H), True))
            # [fw r|u, fw c, bw r|u, bw c] = the bias of the fused input projection
            for d in ("fw", "bw"):
                out.append((f"{pre}/{d}/gru_cell/gates/bias", (2 * H,), True))
                out.append((f"{pre}/{d}/gru_cell/candidate/bias", (H,), True))
        n_in = 2 * H
    out.append(("rnn/logits/kernel", (n_in, cfg.num_classes + 1), True))
    out.append(("rnn/logits/bias", (cfg.num_classes + 1,), True))
    return out


def creation_order(cfg):
    """Variable names in the order the reference graph creates them (what a
    seeded initialiser walks; the buffer order above differs for biases)."""
    names = [n for n, _s, _t in param_shapes(cfg)]
    out = [n for n in names if not n.startswith("rnn/bdrnn")]
    rnn = []
    for li in range(1, len(cfg.rnn_sizes) + 1):
        pre = f"rnn/bdrnn{li}"
        for d in ("fw", "bw"):
            if cfg.cell == "lstm":
                rnn += [f"{pre}/{d}/lstm_cell/kernel", f"{pre}/{d}/lstm_cell/bias"]
            else:
                rnn += [f"{pre}/{d}/gru_cell/{v}" for v in
                        ("gates/kernel", "gates/bias", "candidate/kernel", "candidate/bias")]
    i = out.index("rnn/logits/kernel")
    return out[:i] + rnn + out[i:]


def _trunc_normal(rng, shape, std):
    """[TF1] truncated_normal: redraw values beyond two standard deviations."""
    x = rng.standard_normal(shape)
    bad = np.abs(x) > 2
    while bad.any():
        x[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(x) > 2
    return x * std


def reference_init(cfg, seed=0):
    """Initial values with the reference's initialisers (numpy, host):
    conv + logits kernels: contrib variance_scaling_initializer() -> truncated
    normal, std sqrt(1.3*2/fan_in) (model.py:94, :207); biases 0; BN gamma 1,
    beta 0, moving mean 0 / variance 1; LSTM kernels truncated normal 0.01,
    bias 0 (model_bu.py:170-180); GRU kernels and biases truncated normal 0.01
    (model.py:170-180)."""
    rng = np.random.default_rng(seed)
    vals = {}
    shapes = {n: sh for n, sh, _t in param_shapes(cfg)}
    for name in creation_order(cfg):
        shape = shapes[name]
        leaf = name.rsplit("/", 1)[1]
        if name.startswith("convnet") and leaf == "kernel":
            v = _trunc_normal(rng, shape, np.sqrt(2.6 / (shape[0] * shape[1] * shape[2])))
        elif name == "rnn/logits/kernel":
            v = _trunc_normal(rng, shape, np.sqrt(2.6 / shape[0]))
        elif "gru_cell" in name or ("lstm_cell" in name and leaf == "kernel"):
            v = _trunc_normal(rng, shape, 0.01)
        elif leaf in ("gamma", "moving_variance"):
            v = np.ones(shape)
        else:
            v = np.zeros(shape)
        vals[name] = v.astype(np.float32)
    return vals


class ParamStore:
    def __init__(self, cfg=None, device="cuda", seed=0, values=None):
        self.cfg = cfg or ModelConfig()
        self.device = torch.device(device)
        self.spec = param_shapes(self.cfg)
        self.offsets = {}
        sizes = {True: 0, False: 0}
        for name, shape, tr in self.spec:
            n = int(np.prod(shape))
            self.offsets[name] = (tr, sizes[tr], shape)
            sizes[tr] += (n + _ALIGN - 1) // _ALIGN * _ALIGN
        self.n_trainable = sum(int(np.prod(s)) for _, s, tr in self.spec if tr)
        self.flat = torch.zeros(sizes[True], dtype=torch.float32, device=self.device)
        self.flat_grad = torch.zeros_like(self.flat)
        self.flat_stats = torch.zeros(max(sizes[False], _ALIGN), dtype=torch.float32, device=self.device)
        self.params, self.grads, self.stats = {}, {}, {}
        for name, shape, tr in self.spec:
            _, off, _ = self.offsets[name]
            n = int(np.prod(shape))
            if tr:
                self.params[name] = self.flat[off:off + n].view(shape)
                self.grads[name] = self.flat_grad[off:off + n].view(shape)
            else:
                self.stats[name] = self.flat_stats[off:off + n].view(shape)
        self.version = 0
        self._images = {}
        self.pending = []          # events of side-stream gradient work not yet joined
        self.conv_late = []        # (launch fn, tensors): conv weight gradients queued for the next side fork
        self.bn_group = None       # SyncBN: the process group TRAIN-mode BatchNorm statistics span
        self.f32_conv_exact = False    # fp32 training: the conv tower on exact f32 products (Trainer)
        self.load_state_dict(values if values is not None else reference_init(self.cfg, seed))

    # ------------------------------------------------------------ state
    def state_dict(self):
        """name -> host numpy array (trainable variables and BN moving stats)."""
        out = {k: v.detach().cpu().numpy().copy() for k, v in self.params.items()}
        out.update({k: v.detach().cpu().numpy().copy() for k, v in self.stats.items()})
        return out

    def load_state_dict(self, values):
        for name, _shape, _tr in self.spec:
            if name not in values:
                raise KeyError(f"missing variable {name}")
            dst = self.params.get(name, self.stats.get(name))
            src = torch.as_tensor(np.asarray(values[name], dtype=np.float32))
            if tuple(src.shape) != tuple(dst.shape):
                raise ValueError(f"{name}: shape {tuple(src.shape)} != {tuple(dst.shape)}")
            dst.copy_(src.to(self.device))
        self.bump()

    def save(self, path):
        np.savez(path, **{k.replace("/", "__"): v for k, v in self.state_dict().items()})

    def load(self, path):
        with np.load(path, allow_pickle=False) as z:
            self.load_state_dict({k.replace("__", "/"): z[k] for k in z.files})

    def zero_grad(self):
        self.join()
        self.flat_grad.zero_()

    def join(self):
        """Make the current stream wait for side-stream gradient work
        (model.side_work) so flat_grad is complete in stream order."""
        while self.conv_late:       # queued conv weight gradients no later fork took: inline, in order
            fn, _tensors = self.conv_late.pop(0)
            fn()
        if self.pending:
            cur = torch.cuda.current_stream(self.device)
            for ev in self.pending:
                K.wait_mark(cur, ev)
            self.pending.clear()

    def bump(self):
        """The master values changed: derived weight images are stale."""
        self.version += 1
        self._images.clear()
        self._plan_fresh = False

    # ---------------------------------------------------- weight images
    def images(self, key, builder):
        """Compute-dtype weight layouts, rebuilt once per parameter version. The
        model's images in its compute dtype are stable buffers refreshed together
        by ONE batched launch (ocrk_copy_batch, the job table built once);
        other keys fall back to `builder`."""
        plan = self._plan_for(key)
        if plan is not None:
            if not self._plan_fresh:
                K.copy_batch(plan["table"], plan["njobs"], plan["tiles"], self.flat)
                self._plan_fresh = True
            return plan["images"][key]
        img = self._images.get(key)
        if img is None:
            img = builder()
            self._images[key] = img
        return img

    def _plan_for(self, key):
        if self.device.type != "cuda":
            return None
        dtype = key[-1]
        if dtype != self.cfg.dtype:
            return None
        plan = getattr(self, "_plan", None)
        if plan is None:
            plan = self._plan = self._build_plan(dtype)
            self._plan_fresh = False
        return plan if key in plan["images"] else None

    def _build_plan(self, dtype):
        """Allocate every weight image once and the copy-job table (rows of
        src, dst, rows, cols, in_rs, out_rs, first tile, transpose | dtype << 32)."""
        dev = self.device
        esz = torch.empty(0, dtype=dtype).element_size()
        code = K.dtype_code(dtype)
        jobs, images = [], {}

        def job(src, s_off, rows, cols, in_rs, dst, d_off, out_rs, transpose):
            jobs.append([src.data_ptr() + 4 * s_off, dst.data_ptr() + esz * d_off, rows, cols, in_rs, out_rs, 0,
                         int(transpose) | (code << 32)])

        for li in range(2, 9):
            w = self.params[f"convnet/conv{li}/kernel"]                      # [3][3][Cin][Cout]
            kh, kw, cin, cout = w.shape
            w_nk = torch.empty(cout, kh * kw * cin, dtype=dtype, device=dev)
            w_bwd = torch.empty(cin, kh * kw * cout, dtype=dtype, device=dev)
            job(w, 0, kh * kw * cin, cout, cout, w_nk, 0, kh * kw * cin, True)
            for t in range(kh * kw):
                job(w, t * cin * cout, cin, cout, cout, w_bwd, t * cout, kh * kw * cout, False)
            images[("conv", f"conv{li}", dtype)] = (w_nk, w_bwd)
        for layer in range(1, len(self.cfg.rnn_sizes) + 1):
            pre = f"rnn/bdrnn{layer}"
            if self.cfg.cell == "lstm":
                kf = self.params[f"{pre}/fw/lstm_cell/kernel"]
                rows, G = kf.shape
                H = G // 4
                n_in = rows - H
                wxT = torch.empty(2 * G, n_in, dtype=dtype, device=dev)
                wx = torch.empty(n_in, 2 * G, dtype=dtype, device=dev)
                whT = torch.empty(2, G, H, dtype=dtype, device=dev)
                wh = torch.empty(2, H, G, dtype=dtype, device=dev)
                for d, dn in enumerate(("fw", "bw")):
                    k = self.params[f"{pre}/{dn}/lstm_cell/kernel"]
                    job(k, 0, n_in, G, G, wxT, d * G * n_in, n_in, True)
                    job(k, 0, n_in, G, G, wx, d * G, 2 * G, False)
                    job(k, n_in * G, H, G, G, whT, d * G * H, H, True)
                    job(k, n_in * G, H, G, G, wh, d * H * G, G, False)
                images[("lstm", layer, dtype)] = (wxT, wx, whT, wh, self.flat_bias_pair(layer))
            else:
                gk = self.params[f"{pre}/fw/gru_cell/gates/kernel"]
                rows, G2 = gk.shape
                H = G2 // 2
                n_in = rows - H
                G3 = 3 * H
                wxT = torch.empty(2 * G3, n_in, dtype=dtype, device=dev)
                wx = torch.empty(n_in, 2 * G3, dtype=dtype, device=dev)
                whgT = torch.empty(2, G2, H, dtype=dtype, device=dev)
                whcT = torch.empty(2, H, H, dtype=dtype, device=dev)
                whg = torch.empty(2, H, G2, dtype=dtype, device=dev)
                whc = torch.empty(2, H, H, dtype=dtype, device=dev)
                for d, dn in enumerate(("fw", "bw")):
                    g = self.params[f"{pre}/{dn}/gru_cell/gates/kernel"]
                    c = self.params[f"{pre}/{dn}/gru_cell/candidate/kernel"]
                    job(g, 0, n_in, G2, G2, wxT, d * G3 * n_in, n_in, True)
                    job(c, 0, n_in, H, H, wxT, (d * G3 + G2) * n_in, n_in, True)
                    job(g, 0, n_in, G2, G2, wx, d * G3, 2 * G3, False)
                    job(c, 0, n_in, H, H, wx, d * G3 + G2, 2 * G3, False)
                    job(g, n_in * G2, H, G2, G2, whgT, d * G2 * H, H, True)
                    job(c, n_in * H, H, H, H, whcT, d * H * H, H, True)
                    job(g, n_in * G2, H, G2, G2, whg, d * H * G2, G2, False)
                    job(c, n_in * H, H, H, H, whc, d * H * H, H, False)
                images[("gru", layer, dtype)] = (wxT, wx, whgT, whcT, whg, whc, self.gru_bias_cat(layer))
        lk = self.params["rnn/logits/kernel"]                               # [D][C]
        limg = torch.empty(lk.shape, dtype=dtype, device=dev)
        limgT = torch.empty(lk.shape[1], lk.shape[0], dtype=dtype, device=dev)
        job(lk, 0, lk.shape[0], lk.shape[1], lk.shape[1], limg, 0, lk.shape[1], False)
        job(lk, 0, lk.shape[0], lk.shape[1], lk.shape[1], limgT, 0, lk.shape[0], True)
        images[("logits", dtype)] = limg
        images[("logitsT", dtype)] = limgT
        tiles = 0
        for j in jobs:
            j[6] = tiles
            tiles += -(-j[2] // 32) * -(-j[3] // 32)
        table = torch.tensor(jobs, dtype=torch.int64).to(dev)
        return {"table": table, "njobs": len(jobs), "tiles": tiles, "images": images}

    def conv_images(self, name, dtype):
        """conv2..8: w_nk [Cout][3][3][Cin] (forward), w_bwd [Cin][3][3][Cout]."""
        def build():
            w = self.params[f"convnet/{name}/kernel"]
            kh, kw, cin, cout = w.shape
            w_nk = K.permute3(w, kh * kw * cin, cout, 1, dtype).view(cout, kh * kw * cin)
            w_bwd = K.permute3(w, kh * kw, cin, cout, dtype).view(cin, kh * kw * cout)
            return w_nk, w_bwd
        return self.images(("conv", name, dtype), build)

    def lstm_images(self, layer, dtype):
        """Recurrent layer `layer` (1-based): WxT_cat [8H][In], Wx_cat [In][8H],
        whT [2][4H][H], wh [2][H][4H] in dtype, bias_cat f32 [8H]."""
        def build():
            pre = f"rnn/bdrnn{layer}"
            kf = self.params[f"{pre}/fw/lstm_cell/kernel"]
            rows, G = kf.shape
            H = G // 4
            n_in = rows - H
            dev = kf.device
            wxT = torch.empty(2 * G, n_in, dtype=dtype, device=dev)
            wx = torch.empty(n_in, 2 * G, dtype=dtype, device=dev)
            whT = torch.empty(2, G, H, dtype=dtype, device=dev)
            wh = torch.empty(2, H, G, dtype=dtype, device=dev)
            for d, dn in enumerate(("fw", "bw")):
                k = self.params[f"{pre}/{dn}/lstm_cell/kernel"]
                K.strided_copy(k, n_in, G, G, 1, wxT, 1, n_in, out_offset=d * G * n_in)
                K.strided_copy(k, n_in, G, G, 1, wx, 2 * G, 1, out_offset=d * G)
                K.strided_copy(k, H, G, G, 1, whT, 1, H, out_offset=d * G * H, in_offset=n_in * G)
                K.strided_copy(k, H, G, G, 1, wh, G, 1, out_offset=d * H * G, in_offset=n_in * G)
            bias = self.flat_bias_pair(layer)
            return wxT, wx, whT, wh, bias
        return self.images(("lstm", layer, dtype), build)

    def flat_bias_pair(self, layer):
        """[8H] view over the adjacent fw/bw LSTM biases of `layer`."""
        pre = f"rnn/bdrnn{layer}"
        bf = self.params[f"{pre}/fw/lstm_cell/bias"]
        _, off, _ = self.offsets[f"{pre}/fw/lstm_cell/bias"]
        _, off2, _ = self.offsets[f"{pre}/bw/lstm_cell/bias"]
        n = bf.numel()
        if off2 != off + n:
            raise RuntimeError("LSTM biases must be adjacent in the flat buffer")
        return self.flat[off:off + 2 * n]

    def flat_bias_pair_grad(self, layer):
        pre = f"rnn/bdrnn{layer}"
        _, off, _ = self.offsets[f"{pre}/fw/lstm_cell/bias"]
        n = self.params[f"{pre}/fw/lstm_cell/bias"].numel()
        return self.flat_grad[off:off + 2 * n]

    def gru_images(self, layer, dtype):
        """GRU layer `layer`: WxT_cat [6H][In] and Wx_cat [In][6H] (per direction
        columns r|u|c), whgT [2][2H][H], whcT [2][H][H] (forward), whg [2][H][2H],
        whc [2][H][H] (backward), all in dtype; bias_cat f32 [6H] (a flat view)."""
        def build():
            pre = f"rnn/bdrnn{layer}"
            gk = self.params[f"{pre}/fw/gru_cell/gates/kernel"]
            rows, G2 = gk.shape
            H = G2 // 2
            n_in = rows - H
            G3 = 3 * H
            dev = gk.device
            wxT = torch.empty(2 * G3, n_in, dtype=dtype, device=dev)
            wx = torch.empty(n_in, 2 * G3, dtype=dtype, device=dev)
            whgT = torch.empty(2, G2, H, dtype=dtype, device=dev)
            whcT = torch.empty(2, H, H, dtype=dtype, device=dev)
            whg = torch.empty(2, H, G2, dtype=dtype, device=dev)
            whc = torch.empty(2, H, H, dtype=dtype, device=dev)
            for d, dn in enumerate(("fw", "bw")):
                g = self.params[f"{pre}/{dn}/gru_cell/gates/kernel"]
                c = self.params[f"{pre}/{dn}/gru_cell/candidate/kernel"]
                K.strided_copy(g, n_in, G2, G2, 1, wxT, 1, n_in, out_offset=d * G3 * n_in)
                K.strided_copy(c, n_in, H, H, 1, wxT, 1, n_in, out_offset=(d * G3 + G2) * n_in)
                K.strided_copy(g, n_in, G2, G2, 1, wx, 2 * G3, 1, out_offset=d * G3)
                K.strided_copy(c, n_in, H, H, 1, wx, 2 * G3, 1, out_offset=d * G3 + G2)
                K.strided_copy(g, H, G2, G2, 1, whgT, 1, H, out_offset=d * G2 * H, in_offset=n_in * G2)
                K.strided_copy(c, H, H, H, 1, whcT, 1, H, out_offset=d * H * H, in_offset=n_in * H)
                K.strided_copy(g, H, G2, G2, 1, whg, G2, 1, out_offset=d * H * G2, in_offset=n_in * G2)
                K.strided_copy(c, H, H, H, 1, whc, H, 1, out_offset=d * H * H, in_offset=n_in * H)
            return wxT, wx, whgT, whcT, whg, whc, self.gru_bias_cat(layer)
        return self.images(("gru", layer, dtype), build)

    def _gru_bias_span(self, layer):
        pre = f"rnn/bdrnn{layer}"
        names = [f"{pre}/{d}/gru_cell/{v}" for d in ("fw", "bw") for v in ("gates/bias", "candidate/bias")]
        _, off, _ = self.offsets[names[0]]
        pos = off
        for n in names:
            if self.offsets[n][1] != pos:
                raise RuntimeError("GRU biases must be adjacent in the flat buffer")
            pos += self.params[n].numel()
        return off, pos

    def gru_bias_cat(self, layer):
        """[6H] view: [fw r|u, fw c, bw r|u, bw c] biases of GRU layer `layer`."""
        a, b = self._gru_bias_span(layer)
        return self.flat[a:b]

    def gru_bias_cat_grad(self, layer):
        a, b = self._gru_bias_span(layer)
        return self.flat_grad[a:b]

    def logits_image(self, dtype):
        def build():
            return K.cast(self.params["rnn/logits/kernel"].contiguous(), dtype)
        return self.images(("logits", dtype), build)

    def logits_image_t(self, dtype):
        """[C][D]: the logits weight transposed (the forward GEMM's B_NK operand)."""
        def build():
            return K.cast(self.params["rnn/logits/kernel"].t().contiguous(), dtype)
        return self.images(("logitsT", dtype), build)
