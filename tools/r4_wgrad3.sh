#!/bin/bash
# conv7 / conv8 weight gradients as channel blocks (OCRK_CONV_WGRAD_BLOCKS=2) vs the ping-pong TN engine.
set -o pipefail
out=gpurun_out/wg3
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k wgrad_rows -m gpu > "$out/tests.log" 2>&1 || { tail -n 30 "$out/tests.log"; exit 1; }
tail -n 1 "$out/tests.log"
OCRK_CONV_WGRAD_BLOCKS=2 timeout -k 10 120 python3 tools/bench_wgrad.py > "$out/blocks2.txt" 2>&1 || exit $?
grep conv "$out/blocks2.txt"
bash tools/ab_env.sh wg3 3 "b1:" "b2:OCRK_CONV_WGRAD_BLOCKS=2"
