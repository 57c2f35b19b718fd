#!/bin/bash
# ping-pong GEMM A/B on the step's shapes: default vs persistent long-K vs the deep-lead schedule
set -o pipefail
mkdir -p gpurun_out/pp
{
for rep in 1 2; do
  for cfg in "OCRK_PP_DEEP=0 OCRK_PP_PERSIST_NK=8" "OCRK_PP_DEEP=0 OCRK_PP_PERSIST_NK=64" "OCRK_PP_DEEP=1"; do
    echo "== $cfg"
    env $cfg timeout -k 10 120 python3 -u tools/bench_pp.py --only "L" || exit 1
  done
done
} 2>&1 | tee gpurun_out/pp/ab.txt
