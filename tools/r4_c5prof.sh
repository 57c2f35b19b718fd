#!/bin/bash
# Kernel stats of the C5 serving bench (bucketed fp32 forward + beam-16).
set -o pipefail
out=gpurun_out/c5prof
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c5" -o run --output-format csv -- \
    python3 bench.py --config c5 --steps 4 --warmup 2 > "$out/c5.log" 2>&1 || exit $?
find "$out/c5" -name "*kernel_stats.csv" -exec cp {} "$out/c5_kernel_stats.csv" \;
rm -rf "$out/c5"
