"""TFRecord / tf.train.Example reader without TensorFlow.

Reads the MJSynth word shards the reference trains and evaluates on
(src/weinman/mjsynth.py:337-363 `_read_word_record`; written by
src/weinman/mjsynth-tfrecord.py). Pure Python: the record framing
(uint64 length, masked CRC32C, payload, masked CRC32C) and the protobuf wire
format of Example -> Features -> map<string, Feature>.
"""
import struct

_CRC_TABLE = None


def _crc32c_table():
    global _CRC_TABLE
    if _CRC_TABLE is None:
        tbl = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            tbl.append(c)
        _CRC_TABLE = tbl
    return _CRC_TABLE


_NATIVE = []


def _native_crc():
    """libocrk's host CRC32C (SSE4.2), or None when the library is absent."""
    if not _NATIVE:
        try:
            from . import _lib
            fn = _lib.lib().ocrk_crc32c
            _NATIVE.append(lambda b: int(fn(b, len(b), 0)))
        except Exception:                               # library not built: pure Python
            _NATIVE.append(None)
    return _NATIVE[0]


def crc32c(data):
    data = bytes(data)
    native = _native_crc()
    if native is not None:
        return native(data)
    return crc32c_py(data)


def crc32c_py(data):
    tbl = _crc32c_table()
    c = 0xFFFFFFFF
    for b in data:
        c = tbl[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data):
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def iter_records(path, verify_crc=False):
    """Yield the raw payload of every record in a TFRecord file."""
    with open(path, "rb") as f:
        while True:
            head = f.read(12)
            if not head:
                return
            if len(head) < 12:
                raise ValueError(f"{path}: truncated record header")
            (length,) = struct.unpack("<Q", head[:8])
            data = f.read(length)
            foot = f.read(4)
            if len(data) < length or len(foot) < 4:
                raise ValueError(f"{path}: truncated record")
            if verify_crc:
                if struct.unpack("<I", head[8:])[0] != masked_crc32c(head[:8]):
                    raise ValueError(f"{path}: length CRC mismatch")
                if struct.unpack("<I", foot)[0] != masked_crc32c(data):
                    raise ValueError(f"{path}: data CRC mismatch")
            yield data


def _varint(buf, i):
    shift = result = 0
    while True:
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7


def _fields(buf):
    """Yield (field_number, wire_type, value) of one protobuf message."""
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = buf[i:i + ln]
            i += ln
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fn, wt, v


def _signed64(v):
    return v - (1 << 64) if v >= (1 << 63) else v


def _feature(buf):
    for fn, _wt, v in _fields(buf):
        if fn == 1:                                   # BytesList
            return [bytes(x) for f2, _, x in _fields(v) if f2 == 1]
        if fn == 2:                                   # FloatList (packed or not)
            out = []
            for f2, wt2, x in _fields(v):
                if f2 == 1 and wt2 == 2:
                    out += list(struct.unpack(f"<{len(x) // 4}f", x))
                elif f2 == 1:
                    out.append(struct.unpack("<f", x)[0])
            return out
        if fn == 3:                                   # Int64List (packed or not)
            out = []
            for f2, wt2, x in _fields(v):
                if f2 == 1 and wt2 == 2:
                    j = 0
                    while j < len(x):
                        val, j = _varint(x, j)
                        out.append(_signed64(val))
                elif f2 == 1:
                    out.append(_signed64(x))
            return out
    return []


def parse_example(payload):
    """tf.train.Example bytes -> {feature name: list of values}."""
    feats = {}
    for fn, _wt, v in _fields(payload):
        if fn != 1:
            continue
        for fn2, _, entry in _fields(v):              # Features.feature map entries
            if fn2 != 1:
                continue
            key, val = None, None
            for fn3, _, x in _fields(entry):
                if fn3 == 1:
                    key = bytes(x).decode()
                elif fn3 == 2:
                    val = _feature(x)
            feats[key] = val
    return feats


def read_word_records(path, verify_crc=False):
    """mjsynth._read_word_record (src/weinman/mjsynth.py:337-363) minus the JPEG
    decode: dicts with encoded image bytes, labels, width, text, length, filename."""
    for payload in iter_records(path, verify_crc):
        f = parse_example(payload)
        yield {
            "image": f.get("image/encoded", [b""])[0],
            "labels": list(f.get("image/labels", [])),
            "width": int(f.get("image/width", [1])[0]),
            "filename": f.get("image/filename", [b""])[0].decode(errors="replace"),
            "text": f.get("text/string", [b""])[0].decode(errors="replace"),
            "length": int(f.get("text/length", [1])[0]),
        }
