#!/bin/bash
# conv5 / conv6 weight gradients as row-walk channel blocks: parity, standalone, step A/B;
# the logits forward on 64 x 96 NT tiles rides along.
set -o pipefail
out=gpurun_out/wg2
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -m gpu > "$out/tests.log" 2>&1 || { tail -n 30 "$out/tests.log"; exit 1; }
tail -n 1 "$out/tests.log"
timeout -k 10 120 python3 tools/bench_wgrad.py > "$out/blocks.txt" 2>&1 || exit $?
OCRK_CONV_WGRAD_BLOCKS=0 timeout -k 10 120 python3 tools/bench_wgrad.py > "$out/tn.txt" 2>&1 || exit $?
grep conv "$out/blocks.txt" "$out/tn.txt"
bash tools/ab_env.sh wg 3 "blocks:" "tn:OCRK_CONV_WGRAD_BLOCKS=0"
