"""MI355X-native CNN -> BiLSTM -> CTC line-OCR hot path (drop-in for the
src/weinman graph of tgialoimtr/cnn_lstm_ctc_ocr). Compute runs in libocrk.so
(hand-written HIP for gfx950) behind the C ABI in include/ocrk.h."""
from .config import INFER, TRAIN, ModelConfig  # noqa: F401
from .params import ParamStore  # noqa: F401

__version__ = "0.1.0"
