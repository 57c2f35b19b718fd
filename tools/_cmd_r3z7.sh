set -o pipefail
for r in 0 1; do
bash tools/ab_sched.sh "OCRK_AB=$r" "OCRK_DEFER_DWX=1" "OCRK_DEFER_BIAS=1" "OCRK_CONV_TN4_ITEMS=384" "OCRK_GEMM_NT_STAGED=0" "OCRK_PERSIST_LATE=0" || exit $?
done
