"""The INFER forward of one batch shape captured once as a HIP graph.

The reference evaluates a prebuilt TF graph per batch (validate.py:81-92's
greedy graph, test.py:75-104's loss + decode graph, server.py:80-89's bucket
graphs): one `sess.run` per batch, no per-op host work. Here the forward is
~40 libocrk launches (conv stack, BatchNorm, pooling, two BiLSTM layers, the
logit projection) plus the loss and greedy-decode kernels; launched eagerly
from Python at B=64 the host walk costs as much as the kernels. An InferGraph
captures them ONCE for a fixed (batch, width) on static device buffers and
each batch is one graph launch: `run(image, width)` copies a new batch into
the static buffers (or the caller writes them in place) and replays.

Everything captured is a device kernel on device tensors: the decoders are the
host-sync-free `_raw` forms (dense [B, T] -1 padded + lengths), the CTC loss
runs with check=False (its status bit stays in kernels.status_word for the
caller's next check_status). The graph reads the store's derived weight
images (compute-dtype copies, transposed recurrent weights) cached for the
parameter version it was captured at; a variable update (ParamStore.bump, a
checkpoint restore) makes new images, so replay refuses once the version has
moved -- build a new InferGraph then. The images of the captured version are
held here, so their memory cannot be reused under the graph.
"""
import torch

from . import decode
from .mjsynth import num_classes
from .model import INFER, convnet_layers, ctc_loss_layer, rnn_layers


class InferGraph:
    """Graph-captured INFER forward (+ greedy decode, + CTC loss when `labels`
    are given) of a fixed [batch, 32, width, 1] uint8 shape.

    image / width: static device input buffers to capture on (used in place,
    not copied; default: fresh zero buffers of the given shape). labels: a
    (dense int32 [B, L], lengths int32 [B]) device pair captured in place, or
    None for no loss. decoder: "greedy" (ctc_greedy_decoder_raw) or None.
    After run(): .logits [T, B, C], .seq_len [B], .loss (scalar or None),
    .decoded (i64 [B, T], -1 padded) and .decoded_len (i32 [B]) -- the same
    tensors every replay overwrites."""

    def __init__(self, store, batch=None, width=None, image=None, widths=None, labels=None, decoder="greedy",
                 merge_repeated=True, n_classes=None):
        dev = store.device
        if image is None:
            image = torch.zeros(int(batch), 32, int(width), 1, dtype=torch.uint8, device=dev)
        if widths is None:
            widths = torch.full((image.shape[0],), image.shape[2], dtype=torch.int32, device=dev)
        if image.device != dev or widths.device != dev:
            raise ValueError("InferGraph: static buffers must live on the store's device")
        if decoder not in ("greedy", None):
            raise ValueError("InferGraph: decoder is 'greedy' or None (the beam search runs eagerly beside it)")
        self.store = store
        self.image, self.widths, self.labels = image, widths, labels
        self.decoder, self.merge_repeated = decoder, merge_repeated
        self.n_classes = n_classes or num_classes()
        self.stream = torch.cuda.Stream(dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        # one eager pass on the capture stream creates every lazy resource (workspaces,
        # derived weight images, persistent hand-off words) outside the capture
        with torch.cuda.stream(self.stream):
            self._body()
        self.stream.synchronize()
        self.version = store.version
        self._held = dict(store._images)            # the images the capture reads
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            out = self._body()
        self.logits, self.seq_len, self.loss, self.decoded, self.decoded_len = out
        torch.cuda.current_stream(dev).wait_stream(self.stream)

    def _body(self):
        with torch.no_grad():
            feats, seq = convnet_layers(self.image, self.widths, INFER, self.store)
            logits = rnn_layers(feats, seq, self.n_classes, self.store)
            loss = ctc_loss_layer(logits, self.labels, seq, check=False) if self.labels is not None else None
            dec = dlen = None
            if self.decoder == "greedy":
                dec, dlen, _ = decode.ctc_greedy_decoder_raw(logits, seq, self.merge_repeated)
        return logits, seq, loss, dec, dlen

    def replay(self):
        """One launch of the captured forward on the current static inputs."""
        if self.store.version != self.version:
            raise RuntimeError("InferGraph: the variables changed since capture (ParamStore version "
                               f"{self.version} -> {self.store.version}); build a new InferGraph")
        self.graph.replay()
        return self

    def run(self, image=None, widths=None):
        """Copy a batch of the captured shape (host or device tensors) into the
        static buffers, then replay."""
        if image is not None:
            if tuple(image.shape) != tuple(self.image.shape):
                raise ValueError(f"InferGraph: batch {tuple(image.shape)} != captured {tuple(self.image.shape)}")
            self.image.copy_(image, non_blocking=True)
        if widths is not None:
            self.widths.copy_(torch.as_tensor(widths, dtype=torch.int32), non_blocking=True)
        return self.replay()
