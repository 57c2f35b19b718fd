#!/bin/bash
# Standalone BN layers (tools/bench_bn.py) under a kernel trace: per-kernel averages.
set -o pipefail
out=gpurun_out/bnprof_${1:-x}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/t" -o run --output-format csv -- python3 tools/bench_bn.py \
    > "$out/log.txt" 2>&1 || exit $?
find "$out/t" -name "*kernel_stats.csv" -exec cp {} "$out/stats.csv" \;
rm -rf "$out/t"
grep conv "$out/log.txt"
