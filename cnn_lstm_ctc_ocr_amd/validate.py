"""Drop-in for the inference helpers of src/weinman/validate.py used by the
recognise step (src/processing/server.py:80-89, 134-142)."""
import numpy as np
import torch

from . import kernels as K
from .config import INFER
from .mjsynth import out_charset

mode = INFER   # validate.py:41


def _preprocess_image(image, dtype=torch.float32):
    """validate._preprocess_image (validate.py:56-68): uint8 -> float - 0.5.
    (The train/serve graphs fuse this into the first conv; this standalone op
    exists for callers that want the float image.)"""
    return K.preprocess(image.contiguous(), dtype)


def _get_output(rnn_logits, sequence_length, merge_repeated=True):
    """validate._get_output (validate.py:81-92): ctc_greedy_decoder +
    sparse_tensor_to_dense(default_value=-1). Returns a one-element list
    holding an int64 [B, max_decoded_len] device tensor, like the reference's
    `dts` list."""
    logits = rnn_logits if rnn_logits.dtype == torch.float32 else rnn_logits.float()
    out, out_len, _neg = K.ctc_greedy_decode(logits.contiguous(), sequence_length.to(torch.int32).contiguous(),
                                             merge_repeated)
    width = int(out_len.max().item()) if out_len.numel() else 0
    return [out[:, :width]]


def _get_string(labels):
    """validate._get_string (validate.py:126-129)."""
    return "".join(out_charset[int(c)] for c in labels)


def decode_strings(dense):
    """server.py:134-138: drop the -1 padding and map each row to its string."""
    rows = dense.cpu().numpy() if isinstance(dense, torch.Tensor) else np.asarray(dense)
    return [_get_string([c for c in row if c >= 0]) for row in rows]
