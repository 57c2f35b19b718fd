# OCRK_GEMM_NT_CFG is honoured by the tools-only build only (make exp)
export OCRK_LIB=tools/libocrk_exp.so
set -o pipefail
for c in 6 8 9 10 0 4; do echo "== cfg $c"; OCRK_GEMM_NT_CFG=$c timeout -k 10 100 python tools/bench_gemm.py --only "L2" | grep -v "^total" || exit $?; done
