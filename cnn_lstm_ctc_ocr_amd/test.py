"""Drop-in for the evaluation graph of src/weinman/test.py.

`_get_testing(rnn_logits, sequence_length, label, label_length)` returns the
reference's three scalars (test.py:75-104): the mean CTC loss, label_error =
sum(edit distance of the beam-128 best path) / sum(label_length) (the CER),
and sequence_error = fraction of rows with a non-zero edit distance. All
three stay on the device; the only host sync is none (totals are integer
atomics in the edit-distance kernel).
"""
import torch

from . import decode
from .model import ctc_loss_layer, dense_labels

BEAM_WIDTH = 128       # test.py:86


def _get_testing(rnn_logits, sequence_length, label, label_length=None, beam_width=BEAM_WIDTH, summary=None,
                 step=0):
    """summary: a summary.SummaryWriter that receives loss / label_error /
    sequence_error at `step` (test.py:100-102's tf.summary.scalar calls)."""
    T, B, _ = rnn_logits.shape
    dev = rnn_logits.device
    lab, ln = dense_labels(label, B, dev)
    if label_length is not None:
        ln = label_length.to(device=dev, dtype=torch.int32).contiguous()
    seq_len = sequence_length.to(torch.int32).contiguous()
    with torch.no_grad():
        loss = ctc_loss_layer(rnn_logits.float(), (lab, ln), seq_len)                 # test.py:81
        out, out_len, _ = decode.ctc_beam_search_decoder_raw(rnn_logits, seq_len, beam_width, 1, True)
        totals = torch.zeros(3, dtype=torch.int32, device=dev)
        decode.edit_distance(out[0], out_len[0], lab, ln, totals)                    # test.py:90
    label_error = totals[0].to(torch.float32) / totals[2].to(torch.float32)        # test.py:93-96
    sequence_error = totals[1].to(torch.float32) / B                                 # test.py:97-99
    if summary is not None:
        summary.scalars(step, loss=loss, label_error=label_error, sequence_error=sequence_error)
    return loss, label_error, sequence_error
