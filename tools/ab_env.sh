#!/bin/bash
# Interleaved same-box A/B of the C3 step under environment toggles.
# Usage: bash tools/ab_env.sh TAG REPEATS "name:VAR=v VAR2=v" ...   ("base:" = no toggle)
# (BENCH_ARGS: extra bench.py arguments for every run, e.g. "--dtype fp32")
set -o pipefail
tag=${1:?tag}; reps=${2:?repeats}; shift 2
out=gpurun_out/abe_$tag
mkdir -p "$out"
for r in $(seq 1 "$reps"); do
  for c in "$@"; do
    name=${c%%:*}; envs=${c#*:}
    env $envs timeout -k 10 150 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cer $BENCH_ARGS \
        > "$out/${name}_$r.json" 2> "$out/${name}_$r.err" || exit $?
  done
done
for c in "$@"; do
  name=${c%%:*}
  echo "$name $(for f in "$out/${name}"_*.json; do python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" "$f"; done | tr '\n' ' ')"
done
