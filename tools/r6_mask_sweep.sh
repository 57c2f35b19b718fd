#!/bin/bash
# (Historical: these runs used switches removed from the product in round 6 --
#  SIDE_CU_MASK, FORK_EVENTS, PP_DEEP, ... -- their results are kept under profiles/.)
# The step on its own stream, CU-masked weight-gradient side stream: masks 0/96/128/160/192,
# two passes; then kernel-trace timelines of mask 0 and 128.
set -o pipefail
out=gpurun_out/r6ms; mkdir -p $out
for pass in 1 2; do
  for mask in 0 96 128 160 192; do
    OCRK_SIDE_CU_MASK=$mask timeout -k 10 120 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cer \
        --main-stream own > $out/m${mask}_$pass.json 2> $out/m${mask}_$pass.err || { echo "failed $mask"; exit 1; }
    echo "$pass mask=$mask $(grep -o '"ms_per_step": [0-9.]*' $out/m${mask}_$pass.json)"
  done
done
bash tools/quick_trace.sh r6own0 --main-stream own || exit 1
OCRK_SIDE_CU_MASK=128 bash tools/quick_trace.sh r6own128 --main-stream own; echo "trace rc $?"
