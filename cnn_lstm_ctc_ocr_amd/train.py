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
loss is a batch mean (model.py:228). BatchNorm statistics stay per rank.
"""
import math

import torch
import torch.distributed as dist

from . import kernels as K
from .config import TRAIN
from .model import convnet_layers, ctc_loss_layer, rnn_layers


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
    def __init__(self, store, learning_rate=1e-4, momentum=0.9, decay_rate=0.9, decay_steps=2 ** 16,
                 decay_staircase=False, beta2=0.999, epsilon=1e-8, process_group=None, global_step=0):
        self.store = store
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

    def learning_rate(self, step=None):
        """train.py:120-126 tf.train.exponential_decay."""
        step = self.global_step if step is None else step
        e = step / self.decay_steps
        if self.staircase:
            e = math.floor(e)
        return self.base_lr * self.decay_rate ** e

    def world_size(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group)
        return 1

    def loss_and_grads(self, image, width, label):
        """Forward + backward only; gradients land in store.flat_grad."""
        store = self.store
        store.zero_grad()
        features, seq_len = convnet_layers(image, width, TRAIN, store)
        logits = rnn_layers(features, seq_len, store.cfg.num_classes, store)
        loss = ctc_loss_layer(logits, label, seq_len)
        loss.backward()
        return loss

    def reduce_gradients(self):
        """Sum the flat gradient buffer over the data-parallel ranks (one RCCL
        all-reduce); returns the factor that turns the sum into the mean."""
        self.store.join()
        return allreduce_mean_scale(self.store.flat_grad, self.group)

    def apply_gradients(self):
        store = self.store
        grad_scale = self.reduce_gradients()
        t = self.global_step + 1
        lr = self.learning_rate()
        lr_t = lr * math.sqrt(1 - self.beta2 ** t) / (1 - self.beta1 ** t)
        K.adam_(store.flat, store.flat_grad, self.m, self.v, lr_t, self.beta1, self.beta2, self.eps,
                grad_scale=grad_scale)
        store.bump()
        self.global_step += 1

    def step(self, image, width, label):
        """One training iteration; returns the (device) mean CTC loss."""
        loss = self.loss_and_grads(image, width, label)
        self.apply_gradients()
        return loss
