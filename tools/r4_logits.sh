#!/bin/bash
# Logits forward GEMM (N = 96) tile configurations (experiments library).
set -o pipefail
out=gpurun_out/logits
mkdir -p "$out"
for c in -1 1 2 14 15 16 17 18; do
  OCRK_LIB=tools/libocrk_exp.so OCRK_GEMM_NT_CFG=$c timeout -k 10 60 python3 tools/bench_logits.py >> "$out/cfg.txt" 2>&1 || exit $?
done
grep cfg "$out/cfg.txt"
