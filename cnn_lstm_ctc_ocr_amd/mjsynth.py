"""Character set and input conventions of src/weinman/mjsynth.py."""
import numpy as np

# src/weinman/mjsynth.py:23 (index = label id; blank = len(out_charset))
out_charset = ("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789 "
               "`~!@#$%^&*()-=_+[]{};'\\:\"|,./<>?")


def num_classes():
    """mjsynth.py:25-26."""
    return len(out_charset)


def encode(text):
    """Label ids of a string (mjsynth-tfrecord.py uses out_charset.index)."""
    return [out_charset.index(ch) for ch in text]


def pad_first_row(img_u8):
    """mjsynth._preprocess_image's row duplication (mjsynth.py:191-192), on the
    uint8 image [H, W(, 1)]: 31-row MJSynth crops become 32 rows. The
    float conversion itself is fused into the first conv kernel."""
    return np.concatenate([img_u8[:1], img_u8], axis=0)
