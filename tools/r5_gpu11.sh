#!/bin/bash
# 16-row forward loop: bit-identity / parity tests, model tests, C3 A/B, trace
set -o pipefail
mkdir -p gpurun_out/r5g11
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_persistent.py tests/test_gpu_bf16.py tests/test_gpu_model.py > gpurun_out/r5g11/t.log 2>&1 || { tail -40 gpurun_out/r5g11/t.log; exit 1; }
tail -2 gpurun_out/r5g11/t.log
bash tools/ab_env.sh r5fr16 3 "r16:" "r32:OCRK_LSTM_FWD_R16=0" || exit 1
bash tools/quick_trace.sh r5fr16 || exit 1
grep -E "lstm_fwd" gpurun_out/qt_r5fr16/step_timeline.txt
