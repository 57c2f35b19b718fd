#!/bin/bash
# (Historical: OCRK_IMAGE_SPLIT was measured here and not kept -- profiles/r6_image_split_ab.txt.)
# A/B: the recurrent / logits weight images on a side stream beside the conv
# forward (OCRK_IMAGE_SPLIT=1) vs one launch on the step's stream (0).
# Image-test parity first, then three passes of both arms on one box.
set -o pipefail
out=gpurun_out/r6img; mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_images.py \
    > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for pass in 1 2 3; do
  for split in 1 0; do
    OCRK_IMAGE_SPLIT=$split timeout -k 10 150 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cer \
        --no-trained-cer > $out/s${split}_$pass.json 2> $out/s${split}_$pass.err || { echo "failed $split"; tail -3 $out/s${split}_$pass.err; exit 1; }
    echo "$pass split=$split $(grep -o '"ms_per_step": [0-9.]*' $out/s${split}_$pass.json)"
  done
done
