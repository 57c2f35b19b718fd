#!/bin/bash
# six-product fp32 convs: op + model tests, fp32 step A/B, fp32 trace
set -o pipefail
mkdir -p gpurun_out/r5g9
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_ops.py -k "f32_exact or conv3x3_fwd_bwd" > gpurun_out/r5g9/t_ops.log 2>&1 || { tail -40 gpurun_out/r5g9/t_ops.log; exit 1; }
tail -2 gpurun_out/r5g9/t_ops.log
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 180 --timeout-method thread \
  tests/test_gpu_model.py -k "fp32 or f32" > gpurun_out/r5g9/t_model.log 2>&1 || { tail -40 gpurun_out/r5g9/t_model.log; exit 1; }
tail -2 gpurun_out/r5g9/t_model.log
BENCH_ARGS="--dtype fp32" bash tools/ab_env.sh r5x6 2 "x6:" "f32mfma:OCRK_NT_F32_X6=0" || exit 1
bash tools/quick_trace.sh r5x6 --dtype fp32 || exit 1
head -1 gpurun_out/qt_r5x6/step_timeline.txt
