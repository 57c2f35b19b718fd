"""Drop-in for the width-bucketed recognise service of src/processing/server.py
(Bucket, LocalServer) on the libocrk GPU path.

Semantics kept from the reference:
  * 31 buckets, width ranges (w, w+32] for w = 32, 64, ..., 992 (server.py:63-64);
    a crop is zero-padded (uint8 0, i.e. -0.5 after preprocessing) on the right
    to the bucket's upper width (server.py:29-34);
  * a bucket releases a batch when it holds MORE than batchsize crops or its
    oldest crop waited longer than maxtime (server.py:45);
  * a short batch is topped up with zero crops whose width is widths[0]
    (server.py:123-128); their results are dropped (clientid '-1');
  * one result per crop: (imgid, text) on the client's output queue, text =
    validate._get_string of the -1-filtered labels (server.py:130-141).
Known reference edge cases, reproduced unless fixed deliberately:
  * a crop exactly 32 px wide fits no (w, w+32] bucket; the reference's
    assert(success_count == 1) fails (server.py:114). Here addImage raises
    ValueError; LocalServer(accept_narrow=True) adds a (0, 32] bucket.
  * a 3-channel crop: the reference keeps channel 1 and drops the channel
    axis (server.py:33-35); here channel 1 is kept WITH the axis so the batch
    stays [bs, 32, W, 1].
The model step runs on the GPU: convnet_layers(INFER) -> rnn_layers ->
ctc_greedy_decoder (server.py:83-89), or the beam-search decoder when the
service is built with decoder="beam" (BASELINE config C5, beam 16).
"""
import queue
import time

import numpy as np
import torch

from . import decode, validate
from .config import INFER
from .model import convnet_layers, rnn_layers
from .mjsynth import num_classes

BUCKET_STEP = 32
BUCKET_MAX_WIDTH = 1000


class Bucket:
    """server.py:17-57."""

    def __init__(self, maxtime, batchsize, widthrange):
        self.maxtime = maxtime
        self.batchsize = batchsize
        self.widthrange = widthrange
        self.imgs = []
        self.widths = []
        self.infos = []
        self.oldesttime = None

    def addImgToBucket(self, clientid, imgid, imgtime, img):
        w = img.shape[1]
        if not (self.widthrange[0] < w <= self.widthrange[1]):
            return False
        img = np.asarray(img)
        if img.ndim == 3:
            img = img[:, :, 1:2] if img.shape[2] > 1 else img
        else:
            img = img[:, :, None]
        padded = np.zeros((img.shape[0], self.widthrange[1], 1), np.uint8)
        padded[:, :w] = img
        self.imgs.append(padded)
        self.widths.append(w)
        self.infos.append((clientid, imgid))
        if self.oldesttime is None or imgtime < self.oldesttime:
            self.oldesttime = imgtime
        return True

    def getBatch(self, now=None):
        if not self.imgs:
            return None
        now = time.time() if now is None else now
        if len(self.imgs) > self.batchsize or (now - self.oldesttime) > self.maxtime:
            batch = np.stack(self.imgs[:self.batchsize])
            widths = np.array(self.widths[:self.batchsize], np.int32)
            infos = self.infos[:self.batchsize]
            del self.imgs[:self.batchsize], self.widths[:self.batchsize], self.infos[:self.batchsize]
            self.oldesttime = now          # as the reference (server.py:52)
            return infos, batch, widths
        return None


def fill_batch(infos, batch, widths, bucket_size):
    """server.py:123-128: top a short batch up with zero crops of width widths[0]."""
    n = batch.shape[0]
    if n >= bucket_size:
        return infos, batch, widths
    extra = bucket_size - n
    batch = np.concatenate([batch, np.zeros((extra,) + batch.shape[1:], batch.dtype)])
    widths = np.concatenate([widths, np.full(extra, widths[0], np.int32)])
    return list(infos) + [("-1", "0")] * extra, batch, widths


class Recognizer:
    """The per-batch model step of LocalServer.run (server.py:80-89, 132-138):
    uint8 [bs, 32, W, 1] + widths -> one string per crop. Holds the variables
    (a ParamStore) on one GPU.

    Serving precision: the reference serves in float32, and only a float32
    store gives the reference's strings (greedy and beam decodes are identical
    to the oracle's on the golden MJSynth batch; bf16 differs, CER 0.034 greedy /
    0.022 beam-16 there -- bench.py's cer_vs_ref). A bf16 store is refused
    unless allow_bf16=True states that approximate strings are acceptable."""

    def __init__(self, store, decoder="greedy", beam_width=16, merge_repeated=True, allow_bf16=False,
                 graphs=False):
        if decoder not in ("greedy", "beam"):
            raise ValueError("decoder is 'greedy' or 'beam'")
        if store.cfg.dtype != torch.float32 and not allow_bf16:
            raise ValueError(f"Recognizer: a {store.cfg.dtype} store does not reproduce the reference's strings "
                             "(float32 does); pass allow_bf16=True to serve approximate decodes")
        self.store = store
        self.decoder = decoder
        self.beam_width = beam_width
        self.merge_repeated = merge_repeated
        self.graphs = {} if graphs else None      # (bs, W) -> infer.InferGraph

    def _graphed(self, batch, widths):
        key = tuple(batch.shape)
        g = self.graphs.get(key)
        if g is None or g.version != self.store.version:
            from .infer import InferGraph
            g = self.graphs[key] = InferGraph(self.store, batch=key[0], width=key[2],
                                              decoder="greedy" if self.decoder == "greedy" else None,
                                              merge_repeated=self.merge_repeated)
        return g.run(torch.from_numpy(np.ascontiguousarray(batch, dtype=np.uint8)),
                     torch.from_numpy(np.asarray(widths, np.int32)))

    def labels(self, batch, widths):
        """Dense int64 [bs, max_len] (-1 padded) device tensor. graphs=True: the
        forward of each (bs, W) bucket shape is captured once (infer.InferGraph)
        and replayed per batch."""
        dev = self.store.device
        if self.graphs is not None:
            g = self._graphed(batch, widths)
            if self.decoder == "greedy":
                width = int(g.decoded_len.max().item()) if g.decoded_len.numel() else 0
                return g.decoded[:, :width].clone()
            out, _ = decode.ctc_beam_search_decoder(g.logits, g.seq_len, self.beam_width, 1, self.merge_repeated)
            return out[0]
        with torch.no_grad():
            image = torch.from_numpy(np.ascontiguousarray(batch, dtype=np.uint8)).to(dev, non_blocking=True)
            width = torch.from_numpy(np.asarray(widths, np.int32)).to(dev, non_blocking=True)
            features, seq_len = convnet_layers(image, width, INFER, self.store)
            logits = rnn_layers(features, seq_len, num_classes(), self.store)
            if self.decoder == "greedy":
                return validate._get_output(logits, seq_len, self.merge_repeated)[0]
            out, _ = decode.ctc_beam_search_decoder(logits, seq_len, self.beam_width, 1, self.merge_repeated)
            return out[0]

    def __call__(self, batch, widths):
        return validate.decode_strings(self.labels(batch, widths))


class LocalServer:
    """server.py:59-145. `recognizer` is a Recognizer (or any callable
    (batch, widths) -> list of strings); queues come from `manager` (a
    multiprocessing Manager, or None for in-process queue.Queue)."""

    def __init__(self, recognizer, manager=None, bucket_size=16, bucket_max_time=1.0, accept_narrow=False):
        self.client_inputs = {}
        self.client_outputs = {}
        self.recognizer = recognizer
        self.manager = manager
        self.bucket_size = bucket_size
        self.buckets = [Bucket(bucket_max_time, bucket_size, (w, w + BUCKET_STEP))
                        for w in range(BUCKET_STEP, BUCKET_MAX_WIDTH, BUCKET_STEP)]
        if accept_narrow:
            self.buckets.insert(0, Bucket(bucket_max_time, bucket_size, (0, BUCKET_STEP)))
        self.maxclientid = 0
        self.batches_run = 0
        self._inflight = {}                # batch id -> infos (asynchronous recognizers)
        self._next_batch = 0

    def _queue(self):
        return self.manager.Queue() if self.manager is not None else queue.Queue()

    def register(self):
        clientid = str(self.maxclientid)
        self.maxclientid += 1
        self.client_inputs[clientid] = self._queue()
        self.client_outputs[clientid] = self._queue()
        return clientid, self.client_inputs[clientid], self.client_outputs[clientid]

    def addImage(self, clientid, imgid, imgtime, img):
        hits = sum(b.addImgToBucket(clientid, imgid, imgtime, img) for b in self.buckets)
        if hits != 1:                                   # server.py:114 assert(success_count == 1)
            raise ValueError(f"crop of width {img.shape[1]} fits {hits} buckets (needs exactly 1)")

    def poll_inputs(self, idle_sleep=0.0):
        got = False
        for clientid, q in list(self.client_inputs.items()):
            try:
                imgid, imgtime, img = q.get(block=False)
            except queue.Empty:
                if idle_sleep:
                    time.sleep(idle_sleep)
                continue
            self.addImage(clientid, imgid, imgtime, img)
            got = True
        return got

    def _deliver(self, infos, texts):
        for (clientid, imgid), txt in zip(infos, texts):
            if clientid == "-1":
                continue
            self.client_outputs[clientid].put((imgid, txt), block=False)

    def flush_buckets(self, now=None):
        """Run every bucket that is ready; returns the number of batches run
        (submitted, for an asynchronous recognizer such as ReplicaPool)."""
        n = 0
        for bi, bucket in enumerate(self.buckets):
            b = bucket.getBatch(now)
            if b is None:
                continue
            infos, batch, widths = fill_batch(*b, self.bucket_size)
            if hasattr(self.recognizer, "submit"):
                bid = self._next_batch
                self._next_batch += 1
                self._inflight[bid] = infos
                self.recognizer.submit(bi, bid, batch, widths)
            else:
                self._deliver(infos, self.recognizer(batch, widths))
            n += 1
        self.batches_run += n
        self.collect()
        return n

    def collect(self, block=False):
        """Forward the results an asynchronous recognizer has finished
        (block=True: wait until every submitted batch is back)."""
        if not hasattr(self.recognizer, "poll"):
            return 0
        n = 0
        while self._inflight:
            done = self.recognizer.poll(block=block)
            if not done:
                break
            for bid, texts in done:
                self._deliver(self._inflight.pop(bid), texts)
                n += 1
        return n

    def run(self, states=None, logger=None, stop=None, idle_sleep=0.1):
        """server.py:94-145 main loop; returns when `stop()` is true."""
        if states is not None:
            states["server_started"] = True
        if logger is not None:
            logger.info("server started, waiting image ...")
        while stop is None or not stop():
            try:
                self.poll_inputs(idle_sleep)
                self.flush_buckets()
                self.collect()
            except Exception:
                if logger is None:
                    raise
                logger.exception("SERVER ERROR")


# ------------------------------------------------------- multi-GPU replicas
def _replica_main(rank, device, make_recognizer, inq, outq):
    """Worker process of a ReplicaPool: one recognizer on one device; batches
    in, ("result", batch id, texts) out, until a None item arrives. The
    replica's GPU is made the CURRENT device before anything else, so every
    per-device launch setting of libocrk (kernel LDS limits, CU counts, the
    persistent kernels' co-residency checks) is taken on that GPU and the
    process never initialises cuda:0 by accident."""
    try:
        if isinstance(device, (str, torch.device)) and str(device).startswith("cuda"):
            torch.cuda.set_device(torch.device(device))
        rec = make_recognizer(device)
    except BaseException as e:                       # reported to the pool, which raises
        outq.put(("init_error", rank, f"{type(e).__name__}: {e}"))
        return
    outq.put(("ready", rank, None))
    while True:
        item = inq.get()
        if item is None:
            break
        bid, batch, widths = item
        try:
            outq.put(("result", bid, list(rec(batch, widths))))
        except Exception as e:                        # reported to the server, which raises
            outq.put(("error", bid, f"{type(e).__name__}: {e}"))
    outq.put(("exit", rank, None))


def gpu_recognizer(cfg=None, checkpoint=None, seed=0, decoder="greedy", beam_width=16, allow_bf16=False):
    """A make_recognizer for ReplicaPool: a Recognizer whose ParamStore is
    built on the replica's device (restored from a TF1 checkpoint, or the
    reference initialisers with `seed`). Picklable (spawn)."""
    return _GpuRecognizerFactory(cfg, checkpoint, seed, decoder, beam_width, allow_bf16)


class _GpuRecognizerFactory:
    def __init__(self, cfg, checkpoint, seed, decoder, beam_width, allow_bf16=False):
        self.cfg, self.checkpoint, self.seed, self.decoder, self.beam_width = cfg, checkpoint, seed, decoder, beam_width
        self.allow_bf16 = allow_bf16

    def __call__(self, device):
        from .config import ModelConfig
        from .params import ParamStore
        store = ParamStore(self.cfg or ModelConfig(dtype=torch.float32), device=device, seed=self.seed)
        if self.checkpoint:
            from . import checkpoint as ckpt
            ckpt.restore(store, self.checkpoint)
        return Recognizer(store, decoder=self.decoder, beam_width=self.beam_width, allow_bf16=self.allow_bf16)


class ReplicaError(RuntimeError):
    """A ReplicaPool worker failed to start, died, or raised on a batch."""


class ReplicaPool:
    """Data-parallel recognise step over several GPUs (inference and
    decode are replicas, no exchange), one worker PROCESS per device. The
    LocalServer stays the single bucketing front end (server.py:59-145, with
    the page workers as its clients, ocr-app.py:186-193); each ready batch is
    sent whole to replica (bucket index mod replicas), so a width bucket -- one
    input shape -- always lands on the same GPU. submit / poll make the
    LocalServer asynchronous: batches of different buckets run on their GPUs
    concurrently. `devices`: e.g. ["cuda:0", ..., "cuda:7"].

    Failures surface as ReplicaError naming the replica: a recognizer that
    cannot be built (reported by the worker), a worker process that dies
    (checked while waiting: its exit code), a batch that raised. The reference
    server instead logs and leaves its loop (server.py:144-145) and relies on
    the app's heartbeat watchdog to restart it (ocr-app.py:219-249)."""

    def __init__(self, devices, make_recognizer, start_method="spawn", timeout=600.0):
        import multiprocessing as mp
        ctx = mp.get_context(start_method)
        self.devices = list(devices)
        self.outq = ctx.Queue()
        self.inqs = [ctx.Queue() for _ in self.devices]
        self.procs = [ctx.Process(target=_replica_main, args=(r, d, make_recognizer, self.inqs[r], self.outq),
                                  daemon=True) for r, d in enumerate(self.devices)]
        self.assigned = {}                                   # batch id -> replica (in flight)
        self._pending = []                                   # results collected by a poll() that raised
        self._closed = False
        for pr in self.procs:
            pr.start()
        ready = set()
        deadline = time.time() + timeout
        while len(ready) < len(self.procs):
            msg = self._get(deadline)
            if msg is None:
                self._abort()
                raise ReplicaError(f"replicas {sorted(set(range(len(self.procs))) - ready)} not ready "
                                   f"after {timeout:.0f} s")
            tag, who, info = msg
            if tag == "ready":
                ready.add(who)
            elif tag == "init_error":
                self._abort()
                raise ReplicaError(f"replica {who} ({self.devices[who]}) failed to start: {info}")

    def _dead(self):
        """(rank, exit code) of the first worker that exited, if any."""
        for r, pr in enumerate(self.procs):
            if not pr.is_alive() and pr.exitcode is not None:
                return r, pr.exitcode
        return None

    def _get(self, deadline):
        """Next message, waiting in short slices while checking that every
        worker is alive (None at the deadline)."""
        while True:
            try:
                return self.outq.get(timeout=0.2)
            except queue.Empty:
                pass
            dead = self._dead()
            if dead is not None and not self._closed:
                try:                                         # a message it sent just before exiting
                    return self.outq.get_nowait()
                except queue.Empty:
                    pass
                self._abort()
                raise ReplicaError(f"replica {dead[0]} ({self.devices[dead[0]]}) died with exit code {dead[1]}; "
                                   f"{len(self.assigned)} batches in flight are lost")
            if deadline is not None and time.time() > deadline:
                return None

    def _abort(self):
        self._closed = True
        for pr in self.procs:
            if pr.is_alive():
                pr.terminate()

    def replica_of(self, bucket_index):
        return bucket_index % len(self.procs)

    def submit(self, bucket_index, batch_id, batch, widths):
        dead = self._dead()
        if dead is not None:
            self._abort()
            raise ReplicaError(f"replica {dead[0]} ({self.devices[dead[0]]}) died with exit code {dead[1]}")
        r = self.replica_of(bucket_index)
        self.assigned[batch_id] = r
        self.inqs[r].put((batch_id, np.ascontiguousarray(batch), np.asarray(widths, np.int32)))

    def _take(self, msg, out):
        """File a result into `out`; a batch error is returned (not raised) so
        poll() can keep the results it has already collected."""
        tag, bid, payload = msg
        if tag == "result":
            self.assigned.pop(bid, None)
            out.append((bid, payload))
        elif tag == "error":
            r = self.assigned.pop(bid, None)
            return ReplicaError(f"replica {r} failed on batch {bid}: {payload}")
        return None                                  # control messages ("ready", "exit") carry no batch

    def poll(self, block=False, timeout=600.0):
        """Finished (batch id, texts) pairs (block: wait for at least one).
        A batch that raised in its replica surfaces as ReplicaError; results
        collected by the same poll are not lost -- they are kept and returned
        by the next poll()."""
        out, err = [], None
        pending, self._pending = self._pending, []
        for m in pending:
            err = self._take(m, out) or err
        while err is None:
            try:
                msg = self.outq.get_nowait()
            except queue.Empty:
                if out or not block or not self.assigned:
                    return out
                msg = self._get(time.time() + timeout)
                if msg is None:
                    self._pending = [("result", bid, texts) for bid, texts in out]
                    raise ReplicaError(f"no result from the replicas within {timeout:.0f} s "
                                       f"({len(self.assigned)} batches in flight)")
            err = self._take(msg, out)
        self._pending = [("result", bid, texts) for bid, texts in out]
        raise err

    def close(self):
        self._closed = True
        for q in self.inqs:
            q.put(None)
        for pr in self.procs:
            pr.join(timeout=60)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def predict_signature(store, images, width, beam_width=128, top_paths=3, merge_repeated=False):
    """The serving signature src/weinman/client.py consumes (model 'clreceipt',
    inputs 'images' u8 [bs, 32, W, 1] and 'width' i32 [bs]; client.py:101-123):
    'output0' = beam log-probabilities [bs, top_paths], 'output1'..'output<top_paths>'
    = the decoded paths as dense int64 [bs, len] (-1 padded), from
    ctc_beam_search_decoder(beam_width=128, merge_repeated=False) (client.py:222-233)."""
    dev = store.device
    with torch.no_grad():
        image = torch.as_tensor(np.asarray(images, np.uint8)).to(dev)
        w = torch.as_tensor(np.asarray(width, np.int32)).to(dev)
        features, seq_len = convnet_layers(image, w, INFER, store)
        logits = rnn_layers(features, seq_len, num_classes(), store)
        paths, logp = decode.ctc_beam_search_decoder(logits, seq_len, beam_width, top_paths, merge_repeated)
    out = {"output0": logp.cpu().numpy()}
    for k, p in enumerate(paths, start=1):
        out[f"output{k}"] = p.cpu().numpy()
    return out
