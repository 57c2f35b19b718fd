#!/bin/bash
# (Historical: these runs used switches removed from the product in round 6 --
#  SIDE_CU_MASK, FORK_EVENTS, PP_DEEP, ... -- their results are kept under profiles/.)
# A/B: the step on the NULL stream vs its own non-blocking stream, x the CU-masked
# weight-gradient side stream (OCRK_SIDE_CU_MASK: 0 = off, 192, 224 of 256 CUs).
# Two passes of every arm on one box. Prints ms_per_step per arm.
set -o pipefail
out=gpurun_out/r6ab; mkdir -p $out
for pass in 1 2; do
  for ms in default own; do
    for mask in 0 192 224; do
      OCRK_SIDE_CU_MASK=$mask timeout -k 10 120 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cer \
          --main-stream $ms > $out/${ms}_m${mask}_$pass.json 2> $out/${ms}_m${mask}_$pass.err || { echo "failed $ms $mask"; tail -3 $out/${ms}_m${mask}_$pass.err; exit 1; }
      echo "$pass $ms mask=$mask $(grep -o '"ms_per_step": [0-9.]*' $out/${ms}_m${mask}_$pass.json)"
    done
  done
done
