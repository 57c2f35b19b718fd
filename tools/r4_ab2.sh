#!/bin/bash
# Same-box A/B of hipGraph replay of the C3 forward + backward against eager
# launches (3 x 30 timed steps each).  Usage: bash tools/r4_ab2.sh TAG
set -o pipefail
tag=${1:?tag}
out=gpurun_out/ab2_$tag
mkdir -p "$out"
for r in 1 2 3; do
  for m in eager graph; do
    timeout -k 10 150 python3 bench.py --mode $m --steps 30 --warmup 5 --no-cpu-baseline --no-cer \
        > "$out/${m}_$r.json" 2>"$out/${m}_$r.err" || exit $?
  done
done
for f in "$out"/*_?.json; do echo "$f $(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" "$f")"; done
