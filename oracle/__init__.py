"""CPU oracle for the CNN -> BiLSTM -> CTC hot path -- TEST INFRASTRUCTURE ONLY.

NumPy restatement of the reference graph (src/weinman/model.py, model_bu.py,
validate.py, mjsynth.py, train.py, test.py of tgialoimtr/cnn_lstm_ctc_ocr) and
of the TensorFlow 1.x op semantics it calls. Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this package, and only as the
checker / CPU baseline -- never as the product path.

Pinning (see DESIGN.md "Oracle"): TensorFlow 1.x and Python 2 cannot run in this
container or on the GPU box, so the reference itself cannot be executed. The
oracle is pinned by (1) the reference's own fixtures (the TFRecord shards under
data/: label encoding, widths, sequence lengths), (2) known-answer tests
(brute-force CTC path sums, hand-computed cell steps, greedy/beam merge cases),
and (3) independent implementations in PyTorch CPU where TF1 semantics
coincide (conv, pool, batch norm, LSTM after the gate remap, CTC loss).
"""
