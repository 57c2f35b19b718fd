#!/bin/bash
# masked fp32 conv dgrad on the NT ring: op tests, fp32 model tests, fp32 trace
set -o pipefail
mkdir -p gpurun_out/r5g7
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_ops.py -k "f32_exact or conv3x3_fwd_bwd" > gpurun_out/r5g7/t_ops.log 2>&1 || { tail -40 gpurun_out/r5g7/t_ops.log; exit 1; }
tail -2 gpurun_out/r5g7/t_ops.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread \
  tests/test_gpu_model.py tests/test_gpu_configs.py -k "fp32 or f32" > gpurun_out/r5g7/t_model.log 2>&1 || { tail -40 gpurun_out/r5g7/t_model.log; exit 1; }
tail -2 gpurun_out/r5g7/t_model.log
bash tools/quick_trace.sh r5f32b --dtype fp32 || exit 1
head -1 gpurun_out/qt_r5f32b/step_timeline.txt
