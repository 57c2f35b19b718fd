#!/bin/bash
# Standalone BN backward sweep over the window walk's segment length and channels per thread.
set -o pipefail
out=gpurun_out/bn_sweep
mkdir -p "$out"
: > "$out/sweep.txt"
for nch in 8 4; do
  for seg in 4 8 16; do
    echo "== nch $nch seg $seg" >> "$out/sweep.txt"
    OCRK_BN_ROUTE_NCH=$nch OCRK_BN_ROUTE_SEG=$seg timeout -k 10 120 python3 tools/bench_bn.py 2>&1 | grep -v amdgpu.ids >> "$out/sweep.txt" || exit $?
  done
done
cat "$out/sweep.txt"
