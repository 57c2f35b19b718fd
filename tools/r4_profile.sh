#!/bin/bash
# (Historical: these runs used switches removed from the product in round 6 --
#  SIDE_CU_MASK, FORK_EVENTS, PP_DEEP, ... -- their results are kept under profiles/.)
# Round-4 profiling on the GPU box: kernel stats of the fp32 serving configs
# (C2, C5) and kernel traces of the C3 step with and without the upper layer's
# dW_x deferred behind the lower BPTT (OCRK_DEFER_DWX; d2: also the lowest layer's data
# gradient before its weight gradients, OCRK_DX_FIRST), plus same-box A/B bench lines.  Usage: bash tools/r4_profile.sh TAG
set -o pipefail
tag=${1:?tag}
out=gpurun_out/p_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/c2" -o run --output-format csv -- \
    python3 bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > "$out/c2.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c5" -o run --output-format csv -- \
    python3 bench.py --config c5 --steps 4 --warmup 2 > "$out/c5.log" 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --config c5 --c5-pipeline 0 --steps 4 --warmup 2 > "$out/c5_serial.json" 2>/dev/null || exit $?
timeout -k 10 200 python3 bench.py --config c5 --c5-pipeline 1 --steps 4 --warmup 2 > "$out/c5_pipe.json" 2>/dev/null || exit $?
for d in 0 1 2; do
  export OCRK_DEFER_DWX=$((d >= 1)) OCRK_DX_FIRST=$((d == 2))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c3_d$d" -o run --output-format csv -- \
      python3 bench.py --steps 7 --warmup 3 --no-cpu-baseline --no-cer > "$out/c3_d$d.log" 2>&1 || exit $?
  python3 tools/timeline.py "$(find "$out/c3_d$d" -name '*kernel_trace.csv' | head -1)" > "$out/c3_d${d}_timeline.txt" || exit $?
done
# same-box A/B of the backward issue order and the side-stream item caps
cfgs=("base:" "defer:OCRK_DEFER_DWX=1" "dxfirst:OCRK_DEFER_DWX=1 OCRK_DX_FIRST=1"
      "cap128:OCRK_TN_ITEMS_L1=128 OCRK_CONV_TN_ITEMS=128"
      "dxfirst_cap128:OCRK_DEFER_DWX=1 OCRK_DX_FIRST=1 OCRK_TN_ITEMS_L1=128 OCRK_CONV_TN_ITEMS=128")
unset OCRK_DEFER_DWX OCRK_DX_FIRST
for r in 1 2 3; do
  for c in "${cfgs[@]}"; do
    name=${c%%:*}; envs=${c#*:}
    env $envs timeout -k 10 120 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cer \
        > "$out/ab_${name}_$r.json" 2>/dev/null || exit $?
  done
done
for f in "$out"/ab_*.json; do echo "$f $(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" "$f")"; done
