#!/bin/bash
# Closing bench lines of the round at HEAD: the default line (as the driver runs it)
# and the other configurations, into gpurun_out/lines/.
set -o pipefail
out=gpurun_out/lines; mkdir -p $out
timeout -k 10 400 python3 bench.py > $out/bench_final.json 2> $out/bench_final.err || { tail -5 $out/bench_final.err; exit 1; }
echo "default $(grep -o '"ms_per_step": [0-9.]*' $out/bench_final.json)"
timeout -k 10 200 python3 bench.py --cell gru --steps 30 --no-cpu-baseline --no-cer --no-trained-cer > $out/bench_gru.json 2> $out/bench_gru.err || exit 1
timeout -k 10 200 python3 bench.py --config c2 --steps 30 --no-cpu-baseline --no-cer --no-trained-cer > $out/bench_c2.json 2> $out/bench_c2.err || exit 1
timeout -k 10 200 python3 bench.py --config c5 --no-cpu-baseline --no-cer --no-trained-cer > $out/bench_c5.json 2> $out/bench_c5.err || exit 1
timeout -k 10 200 python3 bench.py --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-cer --no-trained-cer > $out/bench_fp32.json 2> $out/bench_fp32.err || exit 1
for f in gru c2 c5 fp32; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $out/bench_$f.json)"; done
