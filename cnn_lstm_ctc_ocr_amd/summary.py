"""JSONL scalar summaries: the tf.summary.scalar stream of the reference
(`learning_rate` in train.py:139; `loss`, `label_error`, `sequence_error` in
test.py:100-102; TensorBoard target, Makefile:26-27) written as one JSON object
per line -- {"step": s, "tag": value, ..., "wall_time": t} -- so a run can be
followed with `tail -f` / pandas instead of TensorBoard.

Device scalars are never read synchronously: `SummaryWriter.scalars` queues a
non-blocking copy of every tensor value into pinned host memory behind an
event, and a line is written once its event has completed (`flush()` on the
next call, `close()` waits). The hot loop therefore gets no extra sync.
Under data parallelism only rank 0 writes (pass `rank`).
"""
import collections
import json
import os
import time

import torch


class SummaryWriter:
    def __init__(self, path, rank=0):
        self.path = path
        self.enabled = rank == 0
        self._fh = None
        self._pending = collections.deque()          # (event or None, step, {tag: value|pinned tensor}, wall)
        if self.enabled:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
            self._fh = open(path, "a", buffering=1)

    def scalars(self, step, **values):
        """Record scalars for `step`; values may be numbers, 0-d / 1-element
        tensors (device tensors are copied without a sync) or zero-argument
        callables evaluated once the record's device work has landed (e.g. a
        rate from two timing events recorded before this call)."""
        if not self.enabled:
            return
        host, ev = {}, None
        for tag, v in values.items():
            if isinstance(v, torch.Tensor):
                if v.is_cuda:
                    buf = torch.empty(1, dtype=torch.float64, pin_memory=True)
                    buf.copy_(v.detach().reshape(1).to(torch.float64), non_blocking=True)
                    host[tag] = buf
                    if ev is None:
                        ev = torch.cuda.Event()
                else:
                    host[tag] = float(v.detach().reshape(-1)[0])
            else:
                host[tag] = v
                if callable(v) and ev is None and torch.cuda.is_available():
                    ev = torch.cuda.Event()
        if ev is not None:
            ev.record(torch.cuda.current_stream())
        self._pending.append((ev, int(step), host, time.time()))
        self.flush()

    def flush(self, wait=False):
        """Write every record whose device values have landed (in step order)."""
        while self._pending:
            ev, step, host, wall = self._pending[0]
            if ev is not None:
                if wait:
                    ev.synchronize()
                elif not ev.query():
                    return
            self._pending.popleft()
            rec = {"step": step}
            for tag, v in host.items():
                rec[tag] = float(v[0]) if isinstance(v, torch.Tensor) else (v() if callable(v) else v)
            rec["wall_time"] = round(wall, 6)
            self._fh.write(json.dumps(rec) + "\n")

    def close(self):
        if self._fh is not None:
            self.flush(wait=True)
            self._fh.close()
            self._fh = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def read(path):
    """The records of a JSONL summary file (list of dicts)."""
    with open(path) as fh:
        return [json.loads(line) for line in fh if line.strip()]
