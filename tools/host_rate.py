"""Host issue rate of the C3 train step against the device rate (GPU box): is the
step's Python + launch path keeping ahead of the GPU?  Prints host ms/step (the
loop without a sync) and device ms/step (the loop plus the final drain)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from cnn_lstm_ctc_ocr_amd import ModelConfig, ParamStore  # noqa: E402
from cnn_lstm_ctc_ocr_amd.train import Trainer  # noqa: E402

dev = torch.device("cuda", 0)
store = ParamStore(ModelConfig(dtype=torch.bfloat16), device=dev, seed=0)
tr = Trainer(store)
img, widths, labels = bench.synthetic_batch(np.random.default_rng(1234), 256, 256, 125, dev)
for _ in range(5):
    tr.step(img, widths, labels)
torch.cuda.synchronize()
n = 40
t0 = time.perf_counter()
marks = []
for _ in range(n):
    tr.step(img, widths, labels)
    marks.append(time.perf_counter())
t_host = marks[-1] - t0
torch.cuda.synchronize()
t_dev = time.perf_counter() - t0
gaps = np.diff([t0] + marks) * 1e3
print(f"host issue {1e3 * t_host / n:.3f} ms/step (median {np.median(gaps):.3f}, max {gaps.max():.3f}); "
      f"device {1e3 * t_dev / n:.3f} ms/step; drain after the loop {1e3 * (t_dev - t_host):.2f} ms", flush=True)
