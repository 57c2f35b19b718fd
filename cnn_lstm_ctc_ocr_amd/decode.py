"""TF-named CTC decoders and edit distance on device tensors.

Mirrors the tf.nn / tf calls the reference makes on the hot path:
  * ctc_greedy_decoder       -- src/weinman/validate.py:85-90
  * ctc_beam_search_decoder  -- src/weinman/test.py:84-88 (beam 128),
                                src/weinman/client.py:227-231 (merge_repeated=False)
  * edit_distance            -- src/weinman/test.py:90 (normalize=False)
Sparse outputs are returned dense, -1 padded (what sparse_tensor_to_dense(-1)
gives the reference, validate.py:91-92), plus per-row lengths.
"""
import torch

from . import kernels as K


def _f32(logits):
    return (logits if logits.dtype == torch.float32 else logits.float()).contiguous()


def ctc_greedy_decoder(inputs, sequence_length, merge_repeated=True):
    """Returns ([dense i64 [B, max_len]], neg_sum_logits [B, 1]) like
    tf.nn.ctc_greedy_decoder's (decoded, neg_sum_logits)."""
    out, out_len, neg = K.ctc_greedy_decode(_f32(inputs), sequence_length.to(torch.int32).contiguous(),
                                            merge_repeated)
    width = int(out_len.max().item()) if out_len.numel() else 0
    return [out[:, :width]], neg.unsqueeze(1)


def ctc_greedy_decoder_raw(inputs, sequence_length, merge_repeated=True):
    """The same decode without the host sync for the output width: (out i64
    [B, T] (labels then -1), out_len i32 [B], neg_sum_logits f32 [B])."""
    return K.ctc_greedy_decode(_f32(inputs), sequence_length.to(torch.int32).contiguous(), merge_repeated)


def ctc_beam_search_decoder(inputs, sequence_length, beam_width=100, top_paths=1, merge_repeated=True):
    """Returns (decoded, log_probability): decoded is a list of top_paths
    dense i64 [B, max_len_k] tensors (-1 padded), log_probability f32
    [B, top_paths]."""
    out, out_len, logp = K.ctc_beam_decode(_f32(inputs), sequence_length.to(torch.int32).contiguous(),
                                           beam_width, top_paths, merge_repeated)
    widths = out_len.max(dim=1).values.tolist() if out_len.numel() else [0] * top_paths
    return [out[k, :, :int(widths[k])] for k in range(top_paths)], logp


def ctc_beam_search_decoder_raw(inputs, sequence_length, beam_width=100, top_paths=1, merge_repeated=True):
    """Same search without the host sync for the output width: (out
    [top_paths, B, T], out_len [top_paths, B], log_probability)."""
    return K.ctc_beam_decode(_f32(inputs), sequence_length.to(torch.int32).contiguous(), beam_width,
                             top_paths, merge_repeated)


def edit_distance(hypothesis, hypothesis_len, truth, truth_len, totals=None):
    """tf.edit_distance(normalize=False) row by row: f32 [B]."""
    hyp = hypothesis.to(torch.int64).contiguous()
    lab = truth.to(torch.int32).contiguous()
    if lab.dim() == 1:
        lab = lab.reshape(lab.shape[0], 0)
    return K.edit_distance(hyp, hypothesis_len.to(torch.int32).contiguous(), lab,
                           truth_len.to(torch.int32).contiguous(), totals)
