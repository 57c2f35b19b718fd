set -o pipefail
for r in 0 1 2; do
bash tools/ab_sched.sh "OCRK_AB=$r" "OCRK_CONV_TN4_ITEMS=256" "OCRK_CONV_TN4_ITEMS=256 OCRK_TN_ITEMS_L1=160" "OCRK_TN_ITEMS_L1=160" || exit $?
done
