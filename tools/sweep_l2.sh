set -o pipefail
for c in 6 8 9 10 0 4; do echo "== cfg $c"; OCRK_GEMM_NT_CFG=$c timeout -k 10 100 python tools/bench_gemm.py --only "L2" | grep -v "^total" || exit $?; done
