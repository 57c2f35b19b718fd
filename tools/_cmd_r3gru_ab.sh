set -o pipefail
mkdir -p gpurun_out
for r in 0 1; do
for cfg in "OCRK_AB=$r" "OCRK_TN_ITEMS_L1=256 OCRK_CONV_TN_ITEMS=256" "OCRK_TN_ITEMS_L1=160" "OCRK_TN_ITEMS_L1=256"; do
  env $cfg timeout -k 10 200 python bench.py --cell gru --steps 20 --warmup 5 --no-cpu-baseline --no-cer > gpurun_out/ab.log 2>&1 || exit $?
  echo "gru $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
done
done
