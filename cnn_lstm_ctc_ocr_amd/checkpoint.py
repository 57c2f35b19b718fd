"""TF1 checkpoints (TensorBundle V2: `<prefix>.index` + `<prefix>.data-NNNNN-of-NNNNN`)
without TensorFlow, for the reference's Saver-based restore/save paths
(src/weinman/train.py:152-165 _get_init_pretrained / Saver, validate.py:116-124
_get_init_trained, test.py:106-126 _get_checkpoint).

Format (tensorflow/core/util/tensor_bundle):
  * `.index` is a LevelDB-format SSTable (uncompressed blocks): key "" holds a
    BundleHeaderProto, every other key is a variable name whose value is a
    BundleEntryProto {dtype, shape, shard_id, offset, size, crc32c};
  * `.data-*` shards hold the raw little-endian tensor bytes.
The reference ships no checkpoint, so the reader is pinned by round trips
through the writer below and by hand-built tables in tests/test_checkpoint.py
(parity with files written by TensorFlow itself: unpinned).

Variable names are the reference graph's (convnet/conv1/kernel,
convnet/conv2/batch_norm/moving_mean, rnn/bdrnn1/fw/lstm_cell/kernel,
rnn/bdrnn1/fw/gru_cell/gates/kernel, rnn/logits/bias, ...) -- the same keys
ParamStore uses -- plus the optimizer's slots `<var>/Adam`, `<var>/Adam_1`,
`beta1_power`, `beta2_power` and `global_step`.
"""
import os
import re
import struct

import numpy as np

from .tfrecord import _fields, _varint, masked_crc32c

_MAGIC = 0xDB4775248B80FB57
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
           10: np.bool_, 17: np.uint16, 19: np.float16}
_DTYPE_CODE = {np.dtype(v): k for k, v in _DTYPES.items()}


# ----------------------------------------------------------- protobuf bits
def _enc_varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(fn, wt):
    return _enc_varint((fn << 3) | wt)


def _pb_varint(fn, v):
    return _key(fn, 0) + _enc_varint(v & ((1 << 64) - 1))


def _pb_bytes(fn, b):
    return _key(fn, 2) + _enc_varint(len(b)) + b


def _pb_fixed32(fn, v):
    return _key(fn, 5) + struct.pack("<I", v)


# ------------------------------------------------------------- SSTable read
def _block_entries(block):
    n_restarts = struct.unpack("<I", block[-4:])[0]
    end = len(block) - 4 - 4 * n_restarts
    i, key = 0, b""
    while i < end:
        shared, i = _varint(block, i)
        non_shared, i = _varint(block, i)
        vlen, i = _varint(block, i)
        key = key[:shared] + bytes(block[i:i + non_shared])
        i += non_shared
        yield key, bytes(block[i:i + vlen])
        i += vlen


def _read_block(buf, handle, verify):
    off, i = _varint(handle, 0)
    size, _ = _varint(handle, i)
    block = buf[off:off + size]
    ctype = buf[off + size]
    if ctype != 0:
        raise ValueError("compressed SSTable blocks are not supported (TensorBundle writes them uncompressed)")
    if verify:
        crc = struct.unpack("<I", buf[off + size + 1:off + size + 5])[0]
        if crc != masked_crc32c(bytes(block) + bytes([ctype])):
            raise ValueError("SSTable block checksum mismatch")
    return block


def read_table(path, verify=False):
    """All (key, value) pairs of a LevelDB-format table, in key order."""
    with open(path, "rb") as f:
        buf = memoryview(f.read())
    if len(buf) < 48 or struct.unpack("<Q", buf[-8:])[0] != _MAGIC:
        raise ValueError(f"{path}: not an SSTable (bad magic)")
    footer = buf[-48:-8]
    _, i = _varint(footer, 0)
    _, i = _varint(footer, i)                        # metaindex handle (unused)
    idx_start = i
    _, i = _varint(footer, i)
    _, i = _varint(footer, i)
    index = _read_block(buf, footer[idx_start:i], verify)
    out = []
    for _k, handle in _block_entries(index):
        out += list(_block_entries(_read_block(buf, handle, verify)))
    return out


# ----------------------------------------------------------- bundle read
def _entry(value):
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": None, "slices": False}
    for fn, _wt, v in _fields(value):
        if fn == 1:
            e["dtype"] = v
        elif fn == 2:
            for f2, _, d in _fields(v):
                if f2 == 2:
                    size = 0
                    for f3, _, x in _fields(d):
                        if f3 == 1:
                            size = x
                    e["shape"].append(size)
        elif fn == 3:
            e["shard_id"] = v
        elif fn == 4:
            e["offset"] = v
        elif fn == 5:
            e["size"] = v
        elif fn == 6:
            e["crc32c"] = struct.unpack("<I", v)[0]
        elif fn == 7:
            e["slices"] = True
    return e


def read_bundle(prefix, names=None, verify=False):
    """TensorBundle `prefix` -> {variable name: numpy array}."""
    entries = read_table(prefix + ".index", verify)
    header = dict(entries).get(b"")
    num_shards = 1
    if header is not None:
        for fn, _wt, v in _fields(header):
            if fn == 1:
                num_shards = v
            elif fn == 2 and v != 0:
                raise ValueError("big-endian TensorBundle")
    shards = {}
    out = {}
    for key, value in entries:
        if key == b"":
            continue
        name = key.decode()
        if names is not None and name not in names:
            continue
        e = _entry(value)
        if e["slices"]:
            raise ValueError(f"{name}: partitioned variables are not supported")
        if e["dtype"] not in _DTYPES:
            raise ValueError(f"{name}: unsupported dtype enum {e['dtype']}")
        sid = e["shard_id"]
        if sid not in shards:
            shards[sid] = np.memmap(f"{prefix}.data-{sid:05d}-of-{num_shards:05d}", dtype=np.uint8, mode="r")
        raw = bytes(shards[sid][e["offset"]:e["offset"] + e["size"]])
        if verify and e["crc32c"] is not None and masked_crc32c(raw) != e["crc32c"]:
            raise ValueError(f"{name}: data checksum mismatch")
        out[name] = np.frombuffer(raw, dtype=_DTYPES[e["dtype"]]).reshape(e["shape"]).copy()
    return out


# ----------------------------------------------------------- bundle write
def _block(entries, restart_interval=16):
    body, restarts, last = bytearray(), [], b""
    for n, (k, v) in enumerate(entries):
        shared = 0
        if n % restart_interval == 0:
            restarts.append(len(body))
        else:
            while shared < min(len(k), len(last)) and k[shared] == last[shared]:
                shared += 1
        body += _enc_varint(shared) + _enc_varint(len(k) - shared) + _enc_varint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    body += b"".join(struct.pack("<I", r) for r in restarts) + struct.pack("<I", len(restarts))
    return bytes(body)


def _handle(off, size):
    return _enc_varint(off) + _enc_varint(size)


def write_table(path, entries, block_bytes=4096):
    """Write sorted (key, value) pairs as an uncompressed LevelDB-format table."""
    entries = sorted(entries)
    out = bytearray()
    index = []

    def emit(block):
        off = len(out)
        out.extend(block)
        out.extend(b"\x00" + struct.pack("<I", masked_crc32c(block + b"\x00")))
        return _handle(off, len(block))

    cur, size = [], 0
    for k, v in entries:
        cur.append((k, v))
        size += len(k) + len(v)
        if size >= block_bytes:
            index.append((cur[-1][0], emit(_block(cur))))
            cur, size = [], 0
    if cur:
        index.append((cur[-1][0], emit(_block(cur))))
    meta = emit(_block([]))
    idx = emit(_block(index, restart_interval=1))
    footer = meta + idx
    footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", _MAGIC)
    out.extend(footer)
    with open(path, "wb") as f:
        f.write(out)


def write_bundle(prefix, tensors):
    """{name: array} -> `prefix`.index + `prefix`.data-00000-of-00001."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    header = _pb_varint(1, 1) + _pb_varint(2, 0) + _pb_bytes(3, _pb_varint(1, 1))
    entries = [(b"", header)]
    off = 0
    with open(f"{prefix}.data-00000-of-00001", "wb") as f:
        for name in sorted(tensors):
            a = np.asarray(tensors[name])
            a = a if a.flags.c_contiguous else a.copy(order="C")   # (ascontiguousarray makes scalars 1-D)
            if a.dtype not in _DTYPE_CODE:
                raise ValueError(f"{name}: dtype {a.dtype} has no TF enum here")
            raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
            f.write(raw)
            shape = b"".join(_pb_bytes(2, _pb_varint(1, s)) for s in a.shape)
            e = (_pb_varint(1, _DTYPE_CODE[a.dtype]) + _pb_bytes(2, shape) + _pb_varint(4, off)
                 + _pb_varint(5, len(raw)) + _pb_fixed32(6, masked_crc32c(raw)))
            entries.append((name.encode(), e))
            off += len(raw)
    write_table(prefix + ".index", entries)


# ------------------------------------------------------- checkpoint state
def latest_checkpoint(model_dir):
    """tf.train.get_checkpoint_state(dir).model_checkpoint_path (test.py:106-115):
    the `checkpoint` text file's model_checkpoint_path, relative to model_dir."""
    path = os.path.join(model_dir, "checkpoint")
    if not os.path.exists(path):
        raise RuntimeError("No checkpoint file found")
    with open(path) as f:
        for line in f:
            m = re.match(r'\s*model_checkpoint_path:\s*"(.*)"\s*$', line)
            if m:
                p = m.group(1)
                return p if os.path.isabs(p) else os.path.join(model_dir, p)
    raise RuntimeError("No checkpoint file found")


def write_checkpoint_state(model_dir, prefix):
    with open(os.path.join(model_dir, "checkpoint"), "w") as f:
        rel = os.path.relpath(prefix, model_dir)
        f.write(f'model_checkpoint_path: "{rel}"\nall_model_checkpoint_paths: "{rel}"\n')


# ------------------------------------------------------- store <-> bundle
def restore(store, path, trainer=None, strict=True):
    """Saver.restore into a ParamStore (and a Trainer's Adam slots and
    global_step when given). `path` is a checkpoint prefix or a model dir."""
    prefix = latest_checkpoint(path) if os.path.isdir(path) else path
    t = read_bundle(prefix)
    values = {}
    for name, *_ in store.spec:
        if name in t:
            values[name] = t[name]
        elif strict:
            raise KeyError(f"{prefix}: variable {name} not in checkpoint")
        else:
            values[name] = store.state_dict()[name]
    store.load_state_dict(values)
    if trainer is not None:
        import torch
        m = {n: t[f"{n}/Adam"] for n in store.params if f"{n}/Adam" in t}
        v = {n: t[f"{n}/Adam_1"] for n in store.params if f"{n}/Adam_1" in t}
        for slot, src in ((trainer.m, m), (trainer.v, v)):
            for n, a in src.items():
                _, off, shape = store.offsets[n]
                slot[off:off + a.size].copy_(torch.from_numpy(a.reshape(-1).astype(np.float32)))
        if "global_step" in t:
            trainer.global_step = int(t["global_step"])
    return prefix


def adam_power(beta, updates):
    """TF1 AdamOptimizer's beta_power slot after `updates` updates: created as
    beta (_create_slots) and multiplied by beta in float32 by every _finish."""
    b = np.float32(beta)
    p = np.float32(beta)
    for _ in range(int(updates)):
        p = np.float32(p * b)
    return np.array(p, np.float32)


def save(store, model_dir, global_step=None, trainer=None, name="model.ckpt"):
    """Saver.save(sess, model_dir/name, global_step): variables, BN moving
    statistics, Adam slots when a Trainer is given; updates `checkpoint`.
    With a trainer the step is the trainer's (one source for the global_step
    tensor, the file name and the beta powers); a different explicit
    global_step is refused, since restore() would then apply the wrong Adam
    bias correction."""
    if trainer is not None:
        if global_step is not None and int(global_step) != int(trainer.global_step):
            raise ValueError(f"save: global_step={global_step} but the trainer is at step {trainer.global_step}")
        global_step = trainer.global_step
    global_step = 0 if global_step is None else int(global_step)
    os.makedirs(model_dir, exist_ok=True)
    tensors = dict(store.state_dict())
    tensors["global_step"] = np.array(global_step, np.int64)
    if trainer is not None:
        m, v = trainer.m.cpu().numpy(), trainer.v.cpu().numpy()
        for n, p in store.params.items():
            _, off, shape = store.offsets[n]
            tensors[f"{n}/Adam"] = m[off:off + p.numel()].reshape(shape).copy()
            tensors[f"{n}/Adam_1"] = v[off:off + p.numel()].reshape(shape).copy()
        # TF1 AdamOptimizer creates beta*_power = beta* and multiplies it by
        # beta* in _finish after every update: after t updates it holds beta^(t+1)
        # (float32 products, one per update, as the assign_mul ops form them)
        tensors["beta1_power"] = adam_power(trainer.beta1, trainer.global_step)
        tensors["beta2_power"] = adam_power(trainer.beta2, trainer.global_step)
    prefix = os.path.join(model_dir, f"{name}-{global_step}")
    write_bundle(prefix, tensors)
    write_checkpoint_state(model_dir, prefix)
    return prefix
