"""Localise the ping-pong engine's implicit-GEMM data-gradient mismatch: the
same conv3x3_bwd_data call on the NT engine (product library) and on the
ping-pong engine (experiments library, OCRK_GEMM_PP=2), with / without the
ReLU mask and the fused bias gradient. Run twice: OCRK_LIB unset, then
OCRK_LIB=tools/libocrk_exp.so OCRK_GEMM_PP=2; compares against a float64 reference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnn_lstm_ctc_ocr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(3)
for B, H, W, cin, cout in [(16, 3, 125, 256, 256), (16, 7, 126, 128, 128), (4, 3, 125, 128, 256)]:
    dy = torch.randn(B, H, W, cout, device=dev, generator=g).bfloat16()
    w = (torch.randn(3, 3, cin, cout, device=dev, generator=g) / 30).bfloat16()
    w_bwd = w.permute(2, 0, 1, 3).contiguous().view(cin, 9 * cout)
    mask = torch.randn(B, H, W, cin, device=dev, generator=g).bfloat16()
    ref = torch.nn.functional.conv_transpose2d(dy.double().permute(0, 3, 1, 2),
                                               w.double().permute(2, 3, 0, 1).transpose(0, 1), padding=1)
    ref = ref.permute(0, 2, 3, 1)
    for m in (None, mask):
        for db in (False, True):
            dbias = torch.zeros(cin, device=dev) if db else None
            dx = K.conv3x3_bwd_data(dy, w_bwd, relu_mask=m, dbias=dbias)
            r = ref * (m.double() > 0) if m is not None else ref
            err = ((dx.double() - r).norm() / r.norm()).item()
            bad = (dx.double() - r).abs() > 0.05 * r.abs().max()
            where = bad.nonzero()
            print(f"{B}x{H}x{W} {cin}<-{cout} mask={m is not None} dbias={db}: rel {err:.2e} bad {int(bad.sum())}"
                  + (f" first {where[0].tolist()} last {where[-1].tolist()}" if len(where) else ""), flush=True)
