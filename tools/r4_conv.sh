#!/bin/bash
# Standalone conv layers on the product routes, then implicit GEMM only
# (OCRK_CONV_DIRECT=0) and without the row-walking kernels (OCRK_CONV_ROWS=0).
set -o pipefail
out=gpurun_out/conv
mkdir -p "$out"
timeout -k 10 200 python3 tools/bench_conv.py > "$out/default.txt" 2>&1 || exit $?
OCRK_CONV_DIRECT=0 timeout -k 10 200 python3 tools/bench_conv.py > "$out/nodirect.txt" 2>&1 || exit $?
OCRK_CONV_ROWS=0 timeout -k 10 200 python3 tools/bench_conv.py > "$out/norows.txt" 2>&1 || exit $?
OCRK_CONV_DIRECT=0 OCRK_CONV_ROWS=0 timeout -k 10 200 python3 tools/bench_conv.py > "$out/gemmonly.txt" 2>&1 || exit $?
grep -h "conv\|total" "$out"/default.txt "$out"/nodirect.txt "$out"/norows.txt "$out"/gemmonly.txt
