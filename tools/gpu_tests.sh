#!/bin/bash
# GPU test suite on the box (one process), then a default bench line.
# Usage: bash tools/gpu_tests.sh TAG [pytest -k expression]
set -o pipefail
tag=${1:?tag}
out=gpurun_out/t_$tag
mkdir -p "$out"
k=${2:-}
if [ -n "$k" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$k" > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
else
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
fi
tail -3 "$out/tests.log"
