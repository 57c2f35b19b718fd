#!/bin/bash
# split optimizer update: image/model/dist tests, bench A/B, trace
set -o pipefail
mkdir -p gpurun_out/r5g10
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_images.py tests/test_gpu_model.py tests/test_gpu_dist.py tests/test_gpu_configs.py > gpurun_out/r5g10/t.log 2>&1 || { tail -40 gpurun_out/r5g10/t.log; exit 1; }
tail -2 gpurun_out/r5g10/t.log
bash tools/ab_env.sh r5split 3 "split:" "nosplit:OCRK_SPLIT_UPDATE=0" || exit 1
bash tools/quick_trace.sh r5split || exit 1
head -1 gpurun_out/qt_r5split/step_timeline.txt
