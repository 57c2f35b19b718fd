#!/bin/bash
# Same-box A/B of the default bench step under environment toggles (GPU box,
# repo root):  bash tools/ab_sched.sh "OCRK_TN_ITEMS=256" "OCRK_TN_ITEMS=224" ...
# Each configuration runs 20 timed steps; its ms/step is printed on one line.
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cer > gpurun_out/ab.log 2>&1 || exit $?
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
done
