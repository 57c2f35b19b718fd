set -o pipefail
for r in 0 1; do
bash tools/ab_sched.sh "OCRK_AB=$r" "OCRK_CONV_TN4_ITEMS=256" "OCRK_CONV_TN4_ITEMS=384" "OCRK_TN_ITEMS=224" "OCRK_TN_ITEMS=192" \
  "OCRK_CONV_TN4_ITEMS=256 OCRK_TN_ITEMS_L1=160" || exit $?
done
