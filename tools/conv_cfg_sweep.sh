# OCRK_GEMM_NT_CFG is honoured by the tools-only build only (make exp)
export OCRK_LIB=tools/libocrk_exp.so
set -o pipefail
mkdir -p gpurun_out/sw
for c in -1 0 3 6 7 8 9 10; do
  OCRK_GEMM_NT_CFG=$c timeout -k 10 120 python -u tools/bench_conv.py > gpurun_out/sw/c$c.log 2>&1 || exit $?
done
