#!/bin/bash
# Every bench configuration with bench.py's world-1 queue setting (2) against HIP's
# default (OCRK_HW_QUEUES=4), same box.
set -o pipefail
out=gpurun_out/r6qc; mkdir -p $out
echo "box env GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 200 python3 bench.py "$@" > $out/$name.json 2> $out/$name.err || { echo "failed $name"; tail -3 $out/$name.err; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' $out/$name.json) $(grep -o '"hip_hw_queues": "[^"]*"' $out/$name.json)"
}
for pass in 1 2; do
  run c3_q2_$pass --steps 30 --warmup 5 --no-cpu-baseline --no-cer --no-trained-cer
  OCRK_HW_QUEUES=4 run c3_q4_$pass --steps 30 --warmup 5 --no-cpu-baseline --no-cer --no-trained-cer
done
for arm in q2 q4; do
  if [ $arm = q4 ]; then export OCRK_HW_QUEUES=4; fi
  run gru_$arm --cell gru --steps 30 --warmup 5 --no-cpu-baseline --no-cer --no-trained-cer
  run c2_$arm --config c2 --steps 30 --warmup 5 --no-cpu-baseline --no-cer --no-trained-cer
  run c5_$arm --config c5 --no-cpu-baseline --no-cer --no-trained-cer
  run fp32_$arm --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-cer --no-trained-cer
done
