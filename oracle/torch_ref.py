"""PyTorch-CPU restatement of the reference graph -- the CPU BASELINE leg of
bench.py only (BASELINE.md "CPU-baseline plan": TensorFlow 1.x cannot run
here or on the GPU box, so the reference's CPU path is timed as this
restatement of the same graph on the box's host cores).

Test infrastructure: imported by bench.py's cpu_baseline / C1 legs and by
tests/test_oracle.py, which checks it against the NumPy oracle (ref_model,
pinned as described in DESIGN.md section 4) at a small shape -- so the timed
graph is the oracle's graph. Never part of the product path.

Graph (src/weinman/model_bu.py, the LSTM variant the default bench times;
cell="gru" restates src/weinman/model.py's GRUCell layers for bench --cell gru):
  preprocess x*(1/255)-0.5 (validate.py:56-68) -> 8 x conv3x3 (model.py:84-109,
  layer_params :47-54) with training-mode BatchNorm eps 1e-3 on conv2/4/6/8
  (:118-123) + ReLU + max-pools (:111-116, :145) -> time-major features ->
  2 x bidirectional TF1 LSTMCell (i,j,f,o gates, forget bias 1, :167-199) or
  GRUCell ([r,u] = sig([x,h] Wg + bg); c = tanh([x, r*h] Wc + bc);
  h' = u h + (1-u) c; model.py:167-199, 213-214) ->
  dense + ReLU logits (:216-220) -> tf.nn.ctc_loss mean (:224-229, blank 95)
  -> autograd backward -> TF1 Adam (train.py:101-141).
Sequence-length masking (forward(widths=...)): bidirectional_dynamic_rnn with
sequence_length (model_bu.py:187-192, model.py:152-163 for seq_len =
floor((w-2)/2) - 2): each direction is dynamic_rnn -- for steps s >= len the
output is 0 and the state is carried -- and the backward direction runs on
reverse_sequence(x, len) (the first len steps of a row reversed, the rest in
place) with its outputs reversed back the same way. ctc_loss then uses the same
per-row lengths (model.py:224-229). Without widths every row is full (seq_len =
T): the fast path the CPU baseline times.
"""
import math

import torch
import torch.nn.functional as F

LAYERS = [("conv1", 1, 32, "valid", False), ("conv2", 32, 32, "same", True), ("conv3", 32, 64, "same", False),
          ("conv4", 64, 64, "same", True), ("conv5", 64, 128, "same", False), ("conv6", 128, 128, "same", True),
          ("conv7", 128, 256, "same", False), ("conv8", 256, 256, "same", True)]
POOLS = {"conv2": ((2, 2), (2, 2)), "conv4": ((2, 2), (2, 1)), "conv6": ((2, 2), (2, 1)), "conv8": ((3, 1), (3, 1))}


class _RoundBF16(torch.autograd.Function):
    """Identity whose forward value AND incoming gradient are rounded to bf16:
    what bf16 STORAGE of an activation and of its gradient alone does to an
    otherwise exact (float64) computation (tests/test_gpu_bf16.py bounds)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


class TorchRef:
    """Parameters as torch CPU tensors under the TF variable names (the
    oracle's init_params / the ParamStore layout: kernels HWIO / [in+H, 4H]).
    bf16_storage=True rounds every conv-tower op's output and gradient to bf16
    (conv, BN, ReLU, max-pool), as the product stores them."""

    def __init__(self, params, rnn_sizes=(512, 512), dtype=torch.float32, cell="lstm", bf16_storage=False):
        self.q = _RoundBF16.apply if bf16_storage else (lambda t: t)
        self.rnn_sizes = tuple(rnn_sizes)
        self.cell = cell
        self.dtype = dtype
        self.p = {k: torch.tensor(v, dtype=dtype) for k, v in params.items()}
        self.train_names = [k for k in self.p if not k.endswith(("moving_mean", "moving_variance"))]
        for k in self.train_names:
            self.p[k].requires_grad_(True)
        self.m = {k: torch.zeros_like(self.p[k]) for k in self.train_names}
        self.v = {k: torch.zeros_like(self.p[k]) for k in self.train_names}
        self.step_count = 0
        self.seq_len = None

    def forward(self, img_u8, training=True, widths=None):
        """img_u8 uint8 [B, 32, W, 1] -> logits [T, B, 96]; a floating-point
        image is taken as already preprocessed (the training input pipeline's
        float32 batches, mjsynth.py:185-194: first row duplicated, 0.0 dynamic
        padding). widths ([B] true crop widths): the recurrence is masked by
        seq_len_from_width(widths) (self.seq_len holds it afterwards), else every
        row runs all T steps."""
        p = self.p
        if img_u8.dtype == torch.uint8:
            x = img_u8.permute(0, 3, 1, 2).float() * (1.0 / 255.0) - 0.5      # NCHW, float32 as TF
        else:
            x = img_u8.permute(0, 3, 1, 2).float()
        x = x.to(self.dtype)
        q = self.q
        for name, cin, cout, pad, bn in LAYERS:
            w = p[f"convnet/{name}/kernel"].permute(3, 2, 0, 1)                   # HWIO -> OIHW
            x = q(F.conv2d(x, w, p[f"convnet/{name}/bias"], padding=1 if pad == "same" else 0))
            if bn:
                pre = f"convnet/{name}/batch_norm"
                x = q(F.batch_norm(x, p[pre + "/moving_mean"], p[pre + "/moving_variance"], p[pre + "/gamma"],
                                   p[pre + "/beta"], training=training, momentum=0.01, eps=1e-3))
                x = q(F.max_pool2d(q(F.relu(x)), *POOLS[name]))
            else:
                x = q(F.relu(x))
        h = x[:, :, 0, :].permute(2, 0, 1)                                        # [T, B, 256]
        T, B = h.shape[0], h.shape[1]
        self.seq_len = None
        if widths is not None:
            w = torch.as_tensor(widths, dtype=torch.long).reshape(-1)
            self.seq_len = ((w - 2) // 2 - 2).clamp(0, T)                        # model.py:152-163
            return self._masked_rnn(h, self.seq_len)
        for li, H in enumerate(self.rnn_sizes, start=1):
            outs = []
            for d, rev in (("fw", False), ("bw", True)):
                if self.cell == "gru":
                    outs.append(self._gru_dir(h, f"rnn/bdrnn{li}/{d}/gru_cell/", H, rev))
                    continue
                k = p[f"rnn/bdrnn{li}/{d}/lstm_cell/kernel"]
                b = p[f"rnn/bdrnn{li}/{d}/lstm_cell/bias"]
                n_in = h.shape[2]
                gx = h @ k[:n_in] + b                                             # [T, B, 4H] hoisted
                wh = k[n_in:]
                hs = h.new_zeros(h.shape[1], H)
                cs = h.new_zeros(h.shape[1], H)
                seq = []
                gxt = gx.unbind(0)                      # one UnbindBackward, not T x SelectBackward zero-fills
                for t in (range(h.shape[0] - 1, -1, -1) if rev else range(h.shape[0])):
                    z = gxt[t] + hs @ wh
                    i, j, f, o = z.chunk(4, dim=1)
                    cs = torch.sigmoid(f + 1.0) * cs + torch.sigmoid(i) * torch.tanh(j)
                    hs = torch.sigmoid(o) * torch.tanh(cs)
                    seq.append(hs)
                if rev:
                    seq.reverse()
                outs.append(torch.stack(seq))
            h = torch.cat(outs, dim=2)
        return F.relu(h @ p["rnn/logits/kernel"] + p["rnn/logits/bias"])

    def _masked_rnn(self, h, seq_len):
        """rnn_layers with sequence_length (model_bu.py:187-199 / model.py:187-199):
        per direction, x reversed per row by reverse_sequence for bw, a masked
        dynamic_rnn (output 0 and state carried for s >= len), outputs reversed
        back; then the logits (:216-220)."""
        p = self.p
        T, B = h.shape[0], h.shape[1]
        s_idx = torch.arange(T)[:, None]
        valid = s_idx < seq_len[None, :]                                         # [T, B]
        rev_idx = torch.where(valid, seq_len[None, :] - 1 - s_idx, s_idx)        # reverse_sequence, involution
        for li, H in enumerate(self.rnn_sizes, start=1):
            outs = []
            for d, rev in (("fw", False), ("bw", True)):
                n_in = h.shape[2]
                if rev:
                    xin = h.gather(0, rev_idx[:, :, None].expand(T, B, n_in))
                else:
                    xin = h
                if self.cell == "gru":
                    pre = f"rnn/bdrnn{li}/{d}/gru_cell/"
                    gk, gb = p[pre + "gates/kernel"], p[pre + "gates/bias"]
                    ck, cb = p[pre + "candidate/kernel"], p[pre + "candidate/bias"]
                    gxt = (xin @ gk[:n_in] + gb).unbind(0)
                    cxt = (xin @ ck[:n_in] + cb).unbind(0)
                    hs = h.new_zeros(B, H)
                    seq = []
                    for t in range(T):
                        r, u = torch.sigmoid(gxt[t] + hs @ gk[n_in:]).chunk(2, dim=1)
                        c = torch.tanh(cxt[t] + (r * hs) @ ck[n_in:])
                        hn = u * hs + (1 - u) * c
                        m = valid[t][:, None]
                        seq.append(torch.where(m, hn, torch.zeros_like(hn)))
                        hs = torch.where(m, hn, hs)
                else:
                    k = p[f"rnn/bdrnn{li}/{d}/lstm_cell/kernel"]
                    b = p[f"rnn/bdrnn{li}/{d}/lstm_cell/bias"]
                    gxt = (xin @ k[:n_in] + b).unbind(0)
                    wh = k[n_in:]
                    hs = h.new_zeros(B, H)
                    cs = h.new_zeros(B, H)
                    seq = []
                    for t in range(T):
                        i, j, f, o = (gxt[t] + hs @ wh).chunk(4, dim=1)
                        cn = torch.sigmoid(f + 1.0) * cs + torch.sigmoid(i) * torch.tanh(j)
                        hn = torch.sigmoid(o) * torch.tanh(cn)
                        m = valid[t][:, None]
                        seq.append(torch.where(m, hn, torch.zeros_like(hn)))
                        hs = torch.where(m, hn, hs)
                        cs = torch.where(m, cn, cs)
                out = torch.stack(seq)
                if rev:
                    out = out.gather(0, rev_idx[:, :, None].expand(T, B, H))
                outs.append(out)
            h = torch.cat(outs, dim=2)
        return F.relu(h @ p["rnn/logits/kernel"] + p["rnn/logits/bias"])

    def _gru_dir(self, h, pre, H, rev):
        """One direction of the GRU layer; the input halves of both matmuls hoisted."""
        p = self.p
        n_in = h.shape[2]
        gk, gb = p[pre + "gates/kernel"], p[pre + "gates/bias"]
        ck, cb = p[pre + "candidate/kernel"], p[pre + "candidate/bias"]
        gx = h @ gk[:n_in] + gb                                                  # [T, B, 2H]
        cx = h @ ck[:n_in] + cb                                                  # [T, B, H]
        hs = h.new_zeros(h.shape[1], H)
        seq = []
        gxt, cxt = gx.unbind(0), cx.unbind(0)
        for t in (range(h.shape[0] - 1, -1, -1) if rev else range(h.shape[0])):
            r, u = torch.sigmoid(gxt[t] + hs @ gk[n_in:]).chunk(2, dim=1)
            c = torch.tanh(cxt[t] + (r * hs) @ ck[n_in:])
            hs = u * hs + (1 - u) * c
            seq.append(hs)
        if rev:
            seq.reverse()
        return torch.stack(seq)

    def loss(self, logits, labels, label_len, per_sequence=False):
        """mean over the batch of tf.nn.ctc_loss (blank = C-1, loss not length-normalised)
        over the last forward's seq_len (all T without widths); per_sequence=True: the [B] losses."""
        T, B, _ = logits.shape
        lp = F.log_softmax(logits, dim=2)
        seq = torch.full((B,), T, dtype=torch.long) if self.seq_len is None else self.seq_len
        if per_sequence:
            return F.ctc_loss(lp, labels, seq, label_len, blank=logits.shape[2] - 1, reduction="none")
        return F.ctc_loss(lp, labels, seq, label_len, blank=logits.shape[2] - 1, reduction="sum") / B

    def loss_and_grads(self, img_u8, labels, label_len, widths=None):
        """TRAIN-mode forward + backward without an update: (mean loss, {name: grad},
        per-sequence losses [B], logits [T, B, C]) as numpy float64 / self.dtype."""
        for k in self.train_names:
            self.p[k].grad = None
        logits = self.forward(img_u8, True, widths)
        losses = self.loss(logits, labels, label_len, per_sequence=True)
        loss = losses.sum() / logits.shape[1]
        loss.backward()
        grads = {k: self.p[k].grad.detach().numpy() for k in self.train_names}
        return float(loss.detach()), grads, losses.detach().numpy(), logits.detach().numpy()

    def train_step(self, img_u8, labels, label_len, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8):
        """Forward, backward and one TF1 Adam update; returns the loss."""
        for k in self.train_names:
            self.p[k].grad = None
        loss = self.loss(self.forward(img_u8, True), labels, label_len)
        loss.backward()
        self.step_count += 1
        t = self.step_count
        lr_t = lr * math.sqrt(1 - beta2 ** t) / (1 - beta1 ** t)
        with torch.no_grad():
            for k in self.train_names:
                g = self.p[k].grad
                self.m[k].mul_(beta1).add_(g, alpha=1 - beta1)
                self.v[k].mul_(beta2).addcmul_(g, g, value=1 - beta2)
                self.p[k].sub_(lr_t * self.m[k] / (self.v[k].sqrt() + eps))
        return float(loss.detach())

    def greedy(self, img_u8, widths=None):
        """validate._get_output (validate.py:81-92) on CPU: INFER forward +
        greedy decode (first max, merge repeats, drop blank) over seq_len."""
        with torch.no_grad():
            logits = self.forward(img_u8, training=False, widths=widths)
        best = logits.argmax(dim=2).t()                                           # [B, T]
        lens = [logits.shape[0]] * best.shape[0] if self.seq_len is None else self.seq_len.tolist()
        blank = logits.shape[2] - 1
        out = []
        for row, n in zip(best.tolist(), lens):
            seq, prev = [], -1
            for k in row[:n]:
                if k != blank and k != prev:
                    seq.append(k)
                prev = k
            out.append(seq)
        return out
