#!/bin/bash
# A/B of the hardware queues per process (GPU_MAX_HW_QUEUES: 4 = HIP's default on
# this pool; the step's streams -- main, side, status -- map onto them) for the C3
# step. Two passes of each arm on one box, 30 timed steps each.
set -o pipefail
out=gpurun_out/r6q; mkdir -p $out
for pass in 1 2 3 4; do
  for q in ${QUEUES:-4 2 8}; do
    OCRK_HW_QUEUES=$q GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cer \
        --no-trained-cer > $out/q${q}_$pass.json 2> $out/q${q}_$pass.err || { echo "failed $q"; tail -3 $out/q${q}_$pass.err; exit 1; }
    echo "$pass queues=$q $(grep -o '"ms_per_step": [0-9.]*' $out/q${q}_$pass.json)"
  done
done
