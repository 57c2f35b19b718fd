#!/bin/bash
# measurement overhead of the roofline probes: --probe-every 4 / 10 / 20, C3 bf16
set -o pipefail
out=gpurun_out/abe_r5probe; mkdir -p $out
for r in 1 2 3; do
  for pe in 4 10 20; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cer --probe-every $pe > $out/pe${pe}_$r.json 2> $out/pe${pe}_$r.err || exit 1
  done
done
for pe in 4 10 20; do echo "pe$pe $(for f in $out/pe${pe}_*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['frac'])" $f; done | tr '\n' ' ')"; done
