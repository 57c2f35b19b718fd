#!/bin/bash
# A/B of HIP runtime settings for the C3 step: HIP_FORCE_DEV_KERNARG=1 (kernel
# arguments in device memory) vs the default (host-pinned kernargs).
# Three passes of both arms on one box, 30 timed steps each.
set -o pipefail
out=gpurun_out/r6env; mkdir -p $out
for pass in 1 2 3; do
  for arm in def kern; do
    if [ $arm = kern ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
    timeout -k 10 150 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cer \
        --no-trained-cer > $out/${arm}_$pass.json 2> $out/${arm}_$pass.err || { echo "failed $arm"; tail -3 $out/${arm}_$pass.err; exit 1; }
    echo "$pass $arm $(grep -o '"ms_per_step": [0-9.]*' $out/${arm}_$pass.json)"
  done
done
