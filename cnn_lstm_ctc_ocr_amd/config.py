"""Static description of the reference model (src/weinman/model.py, model_bu.py)."""
from dataclasses import dataclass

import torch

# src/weinman/model.py:47-54 -- Filts, K, Padding, Name, BatchNorm?
LAYER_PARAMS = [[32, 3, "valid", "conv1", False],
                [32, 3, "same", "conv2", True],     # pool
                [64, 3, "same", "conv3", False],
                [64, 3, "same", "conv4", True],     # hpool
                [128, 3, "same", "conv5", False],
                [128, 3, "same", "conv6", True],    # hpool
                [256, 3, "same", "conv7", False],
                [256, 3, "same", "conv8", True]]    # hpool 3

# pool after each BN layer (model.py:136, 139, 142, 145): (kh, kw, sh, sw), 'valid'
POOLS = {"conv2": (2, 2, 2, 2), "conv4": (2, 2, 2, 1), "conv6": (2, 2, 2, 1), "conv8": (3, 1, 3, 1)}

rnn_size = 2 ** 9                   # model.py:56 / model_bu.py (LSTM: 512, 512)
BN_EPS = 1e-3                       # [TF1] tf.layers.batch_normalization defaults
BN_MOMENTUM = 0.99

# learn.ModeKeys (model.py:129)
TRAIN = "train"
INFER = "infer"


@dataclass
class ModelConfig:
    """cell='lstm' with (512, 512) is model_bu.py (the north-star BiLSTM);
    cell='gru' with (512, 256) is model.py."""
    cell: str = "lstm"
    rnn_sizes: tuple = (512, 512)
    num_classes: int = 95
    dtype: torch.dtype = torch.bfloat16

    def __post_init__(self):
        if self.cell not in ("lstm", "gru"):
            raise ValueError(f"unknown cell {self.cell!r}")
        self.rnn_sizes = tuple(self.rnn_sizes)
