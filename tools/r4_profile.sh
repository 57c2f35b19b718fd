#!/bin/bash
# Round-4 profiling on the GPU box: kernel stats of the fp32 serving configs
# (C2, C5) and kernel traces of the C3 step with and without the upper layer's
# dW_x deferred behind the lower BPTT (OCRK_DEFER_DWX), plus same-box A/B bench
# lines of that switch.  Usage: bash tools/r4_profile.sh TAG
set -o pipefail
tag=${1:?tag}
out=gpurun_out/p_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/c2" -o run --output-format csv -- \
    python3 bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > "$out/c2.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c5" -o run --output-format csv -- \
    python3 bench.py --config c5 --steps 4 --warmup 2 > "$out/c5.log" 2>&1 || exit $?
for d in 0 1; do
  OCRK_DEFER_DWX=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c3_d$d" -o run --output-format csv -- \
      python3 bench.py --steps 7 --warmup 3 --no-cpu-baseline --no-cer > "$out/c3_d$d.log" 2>&1 || exit $?
  python3 tools/timeline.py "$(find "$out/c3_d$d" -name '*kernel_trace.csv' | head -1)" > "$out/c3_d${d}_timeline.txt" || exit $?
done
for r in 1 2 3; do
  for d in 0 1; do
    OCRK_DEFER_DWX=$d timeout -k 10 120 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cer \
        > "$out/ab_d${d}_$r.json" 2>/dev/null || exit $?
  done
done
for f in "$out"/ab_*.json; do echo "$f $(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" "$f")"; done
