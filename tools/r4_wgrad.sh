#!/bin/bash
# Standalone conv weight gradients: the product routes, then (experiments
# library) the ping-pong TN engine admitted for Cout = 128 (OCRK_PPTN_NMIN=128).
set -o pipefail
out=gpurun_out/wg
mkdir -p "$out"
timeout -k 10 120 python3 tools/bench_wgrad.py > "$out/default.txt" 2>&1 || exit $?
OCRK_LIB=tools/libocrk_exp.so OCRK_PPTN_NMIN=128 timeout -k 10 120 python3 tools/bench_wgrad.py > "$out/pptn128.txt" 2>&1 || exit $?
cat "$out/default.txt" "$out/pptn128.txt"
