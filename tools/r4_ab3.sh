#!/bin/bash
# Round-4 A/B on one box: the 16-row BPTT against the 32-row gather form (C3
# train step, 2 x 30 timed steps each), graph-replayed C2 / C5 serving against
# eager launches, after the persistent-loop and InferGraph GPU tests.
# Usage: bash tools/r4_ab3.sh TAG
set -o pipefail
tag=${1:?tag}
out=gpurun_out/ab3_$tag
mkdir -p "$out"
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
    tests/test_gpu_persistent.py tests/test_gpu_infer.py > "$out/tests.log" 2>&1 || exit $?
b=(python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cer)
for r in 1 2; do
  timeout -k 10 150 "${b[@]}" > "$out/r16_$r.json" 2> "$out/r16_$r.err" || exit $?
  OCRK_LSTM_BWD_R16=0 timeout -k 10 150 "${b[@]}" > "$out/gat_$r.json" 2> "$out/gat_$r.err" || exit $?
done
for m in graph eager; do
  timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --c2-mode $m > "$out/c2_$m.json" 2> "$out/c2_$m.err" || exit $?
  timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --c5-mode $m > "$out/c5_$m.json" 2> "$out/c5_$m.err" || exit $?
done
for f in "$out"/*.json; do
  echo "$f $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" "$f")"
done
