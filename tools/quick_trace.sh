#!/bin/bash
# One rocprofv3 kernel trace of a short bench run + the step timeline and
# kernel stats (GPU box, repo root):  bash tools/quick_trace.sh <tag> [bench args]
set -o pipefail
tag=${1:?tag}; shift
out=gpurun_out/qt_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-cer "$@" > "$out/trace.log" 2>&1 || exit $?
find "$out/trace" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats.csv" \;
python3 tools/timeline.py "$(find "$out/trace" -name '*kernel_trace.csv' | head -1)" > "$out/step_timeline.txt" || exit $?
rm -rf "$out/trace"
