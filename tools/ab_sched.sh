# A/B of the step under the stream-placement toggles (GPU box, repo root)
set -o pipefail
mkdir -p gpurun_out
for cfg in "OCRK_TN_ITEMS=256" "OCRK_TN_ITEMS=192" "OCRK_TN_ITEMS=256" "OCRK_TN_ITEMS=224"; do
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit $?
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
done
