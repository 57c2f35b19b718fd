#!/bin/bash
# slab sums over four workgroups: bit tests, the step A/B, a bf16 trace
set -o pipefail
mkdir -p gpurun_out/r5g8
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_ops.py -k "slab or colsum or bn" > gpurun_out/r5g8/t_ops.log 2>&1 || { tail -40 gpurun_out/r5g8/t_ops.log; exit 1; }
tail -2 gpurun_out/r5g8/t_ops.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_model.py tests/test_gpu_images.py > gpurun_out/r5g8/t_model.log 2>&1 || { tail -40 gpurun_out/r5g8/t_model.log; exit 1; }
tail -2 gpurun_out/r5g8/t_model.log
bash tools/ab_env.sh r5slab 3 "base:" "off:OCRK_SLAB_ROWS=0" || exit 1
bash tools/quick_trace.sh r5slab || exit 1
