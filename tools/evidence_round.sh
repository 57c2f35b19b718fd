#!/bin/bash
# Round evidence on one GPU box: bench lines (default C3 LSTM with CPU baseline
# and CER, GRU cell, C2, C5), the profile_round kernel stats / PMC traffic /
# conv table, and one step's kernel timeline.  Usage: bash tools/evidence_round.sh r2
set -o pipefail
tag=${1:?tag}
out=gpurun_out/ev_$tag
mkdir -p "$out"
timeout -k 10 300 python3 -u bench.py > "$out/bench.log" 2>&1 || exit $?
grep '^{' "$out/bench.log" | tail -1 > "$out/bench.json"
timeout -k 10 200 python3 -u bench.py --cell gru --no-cpu-baseline > "$out/bench_gru.log" 2>&1 || exit $?
grep '^{' "$out/bench_gru.log" | tail -1 > "$out/bench_gru.json"
timeout -k 10 200 python3 -u bench.py --config c2 --no-cpu-baseline > "$out/bench_c2.log" 2>&1 || exit $?
grep '^{' "$out/bench_c2.log" | tail -1 > "$out/bench_c2.json"
timeout -k 10 300 python3 -u bench.py --config c5 --no-cpu-baseline > "$out/bench_c5.log" 2>&1 || exit $?
grep '^{' "$out/bench_c5.log" | tail -1 > "$out/bench_c5.json"
# the C3 train step at the reference's precision (fp32 store: exact f32 MFMA products)
timeout -k 10 300 python3 -u bench.py --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-cer > "$out/bench_fp32.log" 2>&1 || exit $?
grep '^{' "$out/bench_fp32.log" | tail -1 > "$out/bench_fp32.json"
bash tools/profile_round.sh "$tag" || exit $?
python3 tools/timeline.py "$(find gpurun_out/prof_$tag/trace -name '*kernel_trace.csv' | head -1)" > "$out/step_timeline.txt" || exit $?
