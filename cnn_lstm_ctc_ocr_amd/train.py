"""Drop-in for the training step of src/weinman/train.py.

`Trainer.step(image, width, label)` is one iteration of the reference loop
`sess.run([train_op, global_step])` (train.py:196-199): forward in TRAIN mode
(BatchNorm batch statistics + moving-average UPDATE_OPS, train.py:116-118),
CTC loss (model.py:224-229), backward, and AdamOptimizer(beta1=momentum)
with exponential_decay(1e-4, global_step, 2^16, 0.9) (train.py:120-137).

Data parallel: when torch.distributed is initialised with world_size > 1 the
flat fp32 gradient buffer is summed with ONE all-reduce (RCCL over xGMI on
MI355X, backend "nccl") and the Adam kernel divides by world_size -- the mean
of per-rank means, which equals the global mean for equal shards because the
loss is a batch mean (model.py:228). BatchNorm statistics stay per rank
unless Trainer(sync_bn=True).
"""
import collections
import math
import time

import torch
import torch.distributed as dist

from . import _lib
from . import kernels as K
from . import options
from . import model as _model
from .config import TRAIN
from .model import check_feasible_host, convnet_layers, ctc_loss_layer, dense_labels, host_labels, rnn_layers




class GradBuckets:
    """Bucketed data-parallel gradient all-reduce, in backward order.

    The flat gradient buffer is laid out [conv tower | recurrent + logits]
    (ParamStore: the spec order). The recurrent + logits bucket (88 % of the
    bytes with the LSTM 512/512 model: 9.5 M of 10.7 M values) is complete
    once the recurrent backward has been issued -- its weight-gradient GEMMs
    run on the side stream -- so its all-reduce is started right then, on a
    communication stream that waits for that work, and runs beside the conv
    tower's backward. The conv bucket is all-reduced after the tower's
    backward; finish() makes the current stream wait for both.
    (one bucketed all-reduce after backward, overlapped with the
    conv backward; RCCL over xGMI with backend "nccl".)"""

    def __init__(self, store, group=None, comm=None, force=False):
        """comm: a comm.Communicator (libocrk_comm.so, include/ocrk_comm.h) that
        carries the exchange instead of torch.distributed -- the C-ABI
        all-reduce a host without PyTorch would bind. force: run the whole
        exchange even with one rank (the sum over one rank is the identity), so
        the collective really executes on the comm stream beside the conv
        backward -- the C4 path's ordering, exercised on a one-GPU box."""
        self.store, self.group, self.comm, self.force = store, group, comm, bool(force)
        rnn = [off for name, (tr, off, _s) in store.offsets.items() if tr and name.startswith("rnn/")]
        self.split = min(rnn) if rnn else store.flat_grad.numel()
        self.work = None
        self._stream = None
        self._comm_world = comm.info()[0] if comm is not None else None

    def world(self):
        if self.comm is not None:
            return self._comm_world
        if not (dist.is_available() and dist.is_initialized()):
            return 1
        return dist.get_world_size(self.group)

    def active(self):
        """True when the step exchanges gradients (several ranks, or forced)."""
        return self.world() > 1 or (self.force and (self.comm is not None or
                                                    (dist.is_available() and dist.is_initialized())))

    def _sum_(self, t, async_op=False):
        """SUM all-reduce of t in place on the current stream (RCCL through
        torch.distributed or through the C ABI)."""
        if self.comm is not None:
            self.comm.allreduce_(t)
            return None
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)

    def rnn_ready(self, *_):
        """Start the recurrent bucket's all-reduce (called by the hook on the
        conv tower's output gradient, i.e. after the recurrent backward)."""
        if not self.active() or self.work is not None:
            return
        g = self.store.flat_grad
        if g.is_cuda:
            if self._stream is None:
                self._stream = torch.cuda.Stream(g.device)
            K.fork(self._stream, torch.cuda.current_stream(g.device))
            for ev in self.store.pending:                   # the side-stream weight gradients
                K.wait_mark(self._stream, ev)
            with torch.cuda.stream(self._stream):
                self.work = self._sum_(g[self.split:], async_op=True)
                if self.work is None:                       # the C ABI: stream-ordered, joined in finish()
                    self.work = "stream"
                g.record_stream(self._stream)
        else:
            self.work = self._sum_(g[self.split:], async_op=True)

    def finish(self):
        """After the whole backward (and store.join()): reduce the rest, wait
        for both; returns 1/world (the mean-of-equal-shards factor)."""
        if not self.active():
            return 1.0
        world = self.world()
        g = self.store.flat_grad
        if self.work is None:                               # no hook fired: one flat all-reduce
            self._sum_(g)
        else:
            self._sum_(g[:self.split])
            if self.work == "stream":
                torch.cuda.current_stream(g.device).wait_stream(self._stream)
            else:
                self.work.wait()
            self.work = None
        if g.is_cuda:
            # every rank gets the same device status word (the OR over ranks) for
            # this step, so a device error raises on all ranks at the same step
            # (Trainer.poll_status) instead of one rank raising while its peers
            # block in the next collective
            or_allreduce_status(K.status_word(g.device), self.group, comm=self.comm)
        return 1.0 / world


_STATUS_BITS = {}


def or_allreduce_status(word, group=None, comm=None):
    """OR the int32 status word `word` ([1], a bitmask) over the ranks, in place.
    A MAX all-reduce of the word itself would keep only the numerically largest
    rank's word; instead its 31 bits are spread into a one-hot vector, that is
    MAX-reduced in a separate buffer (comm: the C ABI's SUM, then > 0 -- the same
    OR), and the result is OR-ed back into the word, so every rank's bits -- its
    own included -- survive. Stream-ordered (no host sync)."""
    key = word.device
    if key not in _STATUS_BITS:
        _STATUS_BITS[key] = torch.arange(31, dtype=torch.int32, device=word.device)
    bits = _STATUS_BITS[key]
    vec = torch.bitwise_and(torch.bitwise_right_shift(word, bits), 1)
    if comm is not None:
        comm.allreduce_(vec)
        vec = (vec > 0).to(torch.int32)
    else:
        dist.all_reduce(vec, op=dist.ReduceOp.MAX, group=group)
    word.bitwise_or_(torch.bitwise_left_shift(vec, bits).sum(dtype=torch.int32).view(1))
    return word


def allreduce_mean_scale(flat_grad, group=None):
    """In-place SUM all-reduce of `flat_grad` across the process group (no-op
    for a single process); returns 1/world_size."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1.0
    world = dist.get_world_size(group)
    if world > 1:
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=group)
    return 1.0 / world


class Trainer:
    """Device failures surface as exceptions (TF raises at sess.run):
    * labels given as host data (lists / SparseTensor triples) with host widths
      are checked before any launch -- an infeasible batch raises
      InvalidArgumentError and nothing is updated, exactly as in TF;
    * otherwise the CTC kernel and the persistent recurrent kernels set bits in
      the device status word; every step queues a non-blocking copy of it and
      a later step raises if the copy shows a bit (no sync is added), and
      check_status() synchronises and raises. Unlike TF, the deferred error
      comes AFTER the bad step's update was applied (its infeasible sequences
      contributed zero gradient and +inf loss). Only the bits read are cleared
      (atomic AND-NOT), so errors of steps still in flight are not lost.
    * data parallel (world_size > 1): the word is OR-all-reduced with the
      gradients (or_allreduce_status), and every rank reads the copy of the step `status_lag` (2)
      steps back, waiting for it if needed -- all ranks raise at the same
      step, none is left blocking in a collective."""

    def __init__(self, store, learning_rate=1e-4, momentum=0.9, decay_rate=0.9, decay_steps=2 ** 16,
                 decay_staircase=False, beta2=0.999, epsilon=1e-8, process_group=None, global_step=0,
                 summary=None, summary_every=100, sync_bn=False, comm=None, force_exchange=False):
        """summary: a summary.SummaryWriter; every `summary_every` steps it gets
        learning_rate (train.py:139's tf.summary.scalar), the step's loss and
        the global crops/s since the previous record (no sync: device values
        are copied asynchronously). sync_bn: under data parallelism the
        TRAIN-mode BatchNorm statistics (and the backward's two sums) span all
        ranks' batches -- one small SUM all-reduce per BN layer each way -- so N
        ranks compute the single-device reference's step on the union of their
        batches; off (the default) they stay per rank. comm / force_exchange:
        GradBuckets' C-ABI communicator and its one-rank forced exchange."""
        self.store = store
        self.sync_bn = bool(sync_bn)               # the group is resolved at each step (_bn_group)
        self.summary = summary
        self.summary_every = max(1, int(summary_every))
        self._summary_mark = None
        self.base_lr = learning_rate
        self.beta1 = momentum
        self.beta2 = beta2
        self.eps = epsilon
        self.decay_rate = decay_rate
        self.decay_steps = decay_steps
        self.staircase = decay_staircase
        self.group = process_group
        self.global_step = global_step
        self.m = torch.zeros_like(store.flat)
        self.v = torch.zeros_like(store.flat)
        self._grads_zeroed = False                # flat_grad cleared by the last optimizer pass
        self._status_host = None
        self._status_ev = None
        self._status_stream = None
        self._status_ring = collections.deque()     # data parallel: (event, pinned copy) per step
        self.status_lag = 2
        self.buckets = GradBuckets(store, process_group, comm=comm, force=force_exchange)
        self.overlap_allreduce = True          # start the recurrent bucket mid-backward (GradBuckets)

    def learning_rate(self, step=None):
        """train.py:120-126 tf.train.exponential_decay."""
        step = self.global_step if step is None else step
        e = step / self.decay_steps
        if self.staircase:
            e = math.floor(e)
        return self.base_lr * self.decay_rate ** e

    def _bn_group(self):
        """SyncBN's process group, resolved when a step runs (so a Trainer built
        before init_process_group still synchronises): None without sync_bn or
        outside data parallelism (one process: its statistics are the global ones)."""
        if not self.sync_bn or not (dist.is_available() and dist.is_initialized()):
            return None
        return self.group if self.group is not None else dist.group.WORLD

    def world_size(self):
        if self.buckets.comm is not None:
            return self.buckets.world()
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group)
        return 1

    def loss_and_grads(self, image, width, label):
        """Forward + backward only; gradients land in store.flat_grad. A float32
        store trains its conv tower with exact fp32 products (the fp32 serving
        path's bf16x3 split is within 1e-4 on logits but its ~2^-16 per-product
        error is amplified ~200x into the conv-tower gradients by the BN
        backward) and the recurrent layers and logits on the split (5e-5 on their
        gradients): the persistent fp32 loops and the bf16-rate GEMMs. Option
        F32_TRAIN_EXACT=1: exact products everywhere (the per-step fp32 loops)."""
        store = self.store
        if store.cfg.dtype != torch.float32:
            return self._loss_and_grads(image, width, label)
        if options.get("F32_TRAIN_EXACT"):
            with K.f32_exact():
                return self._loss_and_grads(image, width, label)
        prev, store.f32_conv_exact = store.f32_conv_exact, True
        try:
            return self._loss_and_grads(image, width, label)
        finally:
            store.f32_conv_exact = prev

    def _loss_and_grads(self, image, width, label):
        store = self.store
        # the store is shared (serving, other trainers): this Trainer's SyncBN
        # setting holds for its own forward + backward only
        prev_group, store.bn_group = store.bn_group, self._bn_group()
        try:
            return self._forward_backward(image, width, label)
        finally:
            store.bn_group = prev_group

    def _forward_backward(self, image, width, label):
        store = self.store
        if host_labels(label) and not (isinstance(width, torch.Tensor) and width.is_cuda):
            check_feasible_host(label, width)
        if self._grads_zeroed and not (store.device.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            store.join()             # the last optimizer pass left flat_grad zero (ocrk_adam_ex ZERO_GRAD)
        else:
            store.zero_grad()
        self._grads_zeroed = False
        features, seq_len = convnet_layers(image, width, TRAIN, store)
        if self.overlap_allreduce and features.requires_grad and self.buckets.active() and \
                not (features.is_cuda and torch.cuda.is_current_stream_capturing()):
            features.register_hook(self.buckets.rnn_ready)
        logits = rnn_layers(features, seq_len, store.cfg.num_classes, store)
        loss = ctc_loss_layer(logits, label, seq_len)
        # d loss / d loss = 1 from a resident scalar: no fill launch per step, and the
        # CTC backward skips its x 1 pass over the logits gradient
        if loss.dtype == torch.float32:
            _model.unit_backward(loss)
        else:
            loss.backward()
        return loss

    def reduce_gradients(self):
        """Sum the flat gradient buffer over the data-parallel ranks (RCCL
        all-reduces, the recurrent bucket already started mid-backward);
        returns the factor that turns the sum into the mean."""
        self.store.join()
        return self.buckets.finish()

    def apply_gradients(self):
        store = self.store
        grad_scale = self.reduce_gradients()
        t = self.global_step + 1
        lr = self.learning_rate()
        lr_t = lr * math.sqrt(1 - self.beta2 ** t) / (1 - self.beta1 ** t)
        zero = store.device.type == "cuda"
        # the update clears the gradient as it reads it: the next loss_and_grads skips its fill
        # (a 4-byte-per-parameter pass at the top of the step)
        K.adam_(store.flat, store.flat_grad, self.m, self.v, lr_t, self.beta1, self.beta2, self.eps,
                grad_scale=grad_scale, zero_grad=zero)
        self._grads_zeroed = zero
        store.bump()
        self.global_step += 1

    def step(self, image, width, label):
        """One training iteration; returns the (device) mean CTC loss."""
        self.poll_status()
        lr = self.learning_rate()
        loss = self.loss_and_grads(image, width, label)
        self.apply_gradients()
        self.post_status()
        self.summarize(loss, lr, int(image.shape[0]))
        return loss

    def summarize(self, loss, lr, batch):
        """JSONL scalars every `summary_every` steps (train.py:139).

        The record's step is the post-increment global_step, as TF's summary of
        `sess.run([train_op, global_step])`; `lr` is the rate that step's update
        used (exponential_decay of the pre-increment count) and `loss` its loss.
        crops_per_sec is timed on the DEVICE: an event recorded on the current
        stream at each summary mark, the rate read from the two events' elapsed
        time once the writer's copies have landed (no sync in the loop)."""
        if self.summary is None:
            return
        if self._summary_mark is not None and self.global_step % self.summary_every:
            return                                # events only at the marks (a record costs ~6 us)
        dev = self.store.device
        if dev.type == "cuda":
            now = torch.cuda.Event(enable_timing=True)
            now.record(torch.cuda.current_stream(dev))
        else:
            now = time.perf_counter()
        if self._summary_mark is None:
            self._summary_mark = (self.global_step, now)
        if self.global_step % self.summary_every:
            return
        s0, t0 = self._summary_mark
        crops = (self.global_step - s0) * batch * self.world_size()
        vals = {"learning_rate": lr, "loss": loss}
        if self.global_step > s0:
            if dev.type == "cuda":
                vals["crops_per_sec"] = lambda: round(crops / max(t0.elapsed_time(now) / 1e3, 1e-9), 2)
            elif now > t0:
                vals["crops_per_sec"] = round(crops / (now - t0), 2)
        self.summary.scalars(self.global_step, **vals)
        self._summary_mark = (self.global_step, now)

    # ---- device status word (include/ocrk.h, ocrk_device_status)
    def post_status(self):
        """Queue a non-blocking copy of the device status word (after the step's work)."""
        dev = self.store.device
        if dev.type == "cuda" and self.buckets.active():
            buf = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            buf.copy_(K.status_word(dev), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            self._status_ring.append((ev, buf))
            return
        if dev.type != "cuda" or self._status_ev is not None:
            return
        if self._status_host is None:
            self._status_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._status_stream = torch.cuda.Stream(dev)
        # the copy waits for the step on its own stream: the next step's first kernels
        # do not queue behind it on the main stream
        cur = torch.cuda.current_stream(dev)
        K.fork(self._status_stream, cur)
        with torch.cuda.stream(self._status_stream):
            self._status_host.copy_(K.status_word(dev), non_blocking=True)
            self._status_ev = torch.cuda.Event()
            self._status_ev.record(self._status_stream)

    def poll_status(self):
        """Raise if an earlier step's queued status copy has landed and shows a bit
        (single process: never waits; data parallel: the copy of the step
        `status_lag` steps back, the same step on every rank)."""
        while len(self._status_ring) > self.status_lag:
            ev, buf = self._status_ring.popleft()
            ev.synchronize()
            v = int(buf[0])
            if v:
                self._status_ring.clear()
                K.clear_status(self.store.device, v)
                _lib.raise_for_status(v)
        if self._status_ev is None or not self._status_ev.query():
            return
        v = int(self._status_host[0])
        self._status_ev = None
        if v:
            K.clear_status(self.store.device, v)
            _lib.raise_for_status(v)

    def check_status(self):
        """Synchronise and raise if any step so far set a device status bit."""
        self._status_ev = None
        self._status_ring.clear()
        if self.store.device.type == "cuda":
            K.check_status(self.store.device)

    def graphed(self, image, width, label, max_label_len=None, before_capture=None):
        """A GraphedStep for batches shaped like (image, width, label)."""
        return GraphedStep(self, image, width, label, max_label_len, before_capture)


class GraphedStep:
    """The train step with its forward + backward captured ONCE into a HIP
    graph (torch.cuda.CUDAGraph over the libocrk launches, side-stream weight
    gradients included as graph branches) and replayed for every batch.

    The reference executes a prebuilt dataflow graph per step as well
    (`sess.run([train_op, global_step])`, train.py:196-199); here the graph is
    the ~600 kernel launches of one step, so a step costs one graph launch on
    the host instead of a Python walk over every op. Replays run exactly the
    captured kernels on the static input buffers: `step(image, width, label)`
    copies a new batch (same shape; labels up to `max_label_len`) into them
    first. The gradient all-reduce (world_size > 1) and the Adam launch stay
    eager after the replay, so the learning-rate schedule and RCCL see the live
    host step count.

    Capture needs every per-stream lazy resource (workspaces, kernel
    attributes, hand-off flag words) to exist, so one eager forward + backward runs first on the
    capture stream; the BatchNorm moving statistics it would have updated are
    restored, and gradients are rewritten by every step anyway. The derived
    weight images are invalidated before capture so that their rebuild from
    the live fp32 master values is part of every replay.
    """

    def __init__(self, trainer, image, width, label, max_label_len=None, before_capture=None):
        store = trainer.store
        dev = store.device
        if trainer._bn_group() is not None and trainer.world_size() > 1:
            # SyncBN's collectives sit inside the forward and backward: not captured here
            raise NotImplementedError("GraphedStep with Trainer(sync_bn=True): run eager steps")
        self.trainer = trainer
        self.B = int(image.shape[0])
        self.image = image.detach().to(dev).clone()
        self.width = torch.as_tensor(width).to(device=dev, dtype=torch.int32).clone()
        lab, ln = dense_labels(label, self.B, dev)
        lmax = int(max_label_len or lab.shape[1])
        if lab.shape[1] > lmax:
            raise ValueError(f"labels of {lab.shape[1]} > max_label_len={lmax}")
        self.labels = torch.zeros(self.B, lmax, dtype=torch.int32, device=dev)
        self.labels[:, :lab.shape[1]].copy_(lab)
        self.label_len = ln.clone()
        self.stream = torch.cuda.Stream(dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        moving = store.flat_stats.clone()
        overlap, trainer.overlap_allreduce = trainer.overlap_allreduce, False   # no collective in the warm-up pass
        with torch.cuda.stream(self.stream):
            trainer.loss_and_grads(self.image, self.width, (self.labels, self.label_len))
            store.flat_stats.copy_(moving)
            store.join()
        trainer.overlap_allreduce = overlap
        self.stream.synchronize()
        store.bump()                 # the weight-image rebuilds must be captured, not cache hits
        if before_capture is not None:
            before_capture()         # e.g. drop timers recorded by the eager warm-up
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            self.loss = trainer.loss_and_grads(self.image, self.width, (self.labels, self.label_len))
        torch.cuda.current_stream(dev).wait_stream(self.stream)

    def load(self, image=None, width=None, label=None):
        """Copy a batch into the graph's static input buffers."""
        if image is not None:
            if tuple(image.shape) != tuple(self.image.shape) or image.dtype != self.image.dtype:
                raise ValueError(f"image {tuple(image.shape)} {image.dtype} does not match the captured "
                                 f"{tuple(self.image.shape)} {self.image.dtype}")
            self.image.copy_(image)
        if width is not None:
            self.width.copy_(torch.as_tensor(width).to(device=self.width.device, dtype=torch.int32))
        if label is not None:
            if host_labels(label) and width is not None and not (isinstance(width, torch.Tensor) and width.is_cuda):
                check_feasible_host(label, width)
            lab, ln = dense_labels(label, self.B, self.labels.device)
            if lab.shape[1] > self.labels.shape[1]:
                raise ValueError(f"labels of {lab.shape[1]} > captured max_label_len={self.labels.shape[1]}")
            self.labels.zero_()
            self.labels[:, :lab.shape[1]].copy_(lab)
            self.label_len.copy_(ln)

    def step(self, image=None, width=None, label=None):
        """One training iteration on the given batch (or the loaded one);
        returns the graph's device loss tensor (overwritten by the next step)."""
        self.trainer.poll_status()
        lr = self.trainer.learning_rate()
        self.load(image, width, label)
        self.graph.replay()
        self.trainer.apply_gradients()
        self.trainer.post_status()
        self.trainer.summarize(self.loss, lr, self.B)
        return self.loss
