# OCRK_GEMM_NT_CFG is honoured by the tools-only build only (make exp)
export OCRK_LIB=tools/libocrk_exp.so
set -o pipefail
mkdir -p gpurun_out
OCRK_GEMM_NT=0 timeout -k 10 120 python tools/bench_gemm.py > gpurun_out/bg_old.log 2>&1 || exit $?
for c in 1 6 7 8; do
  OCRK_GEMM_NT=1 OCRK_GEMM_NT_CFG=$c timeout -k 10 120 python tools/bench_gemm.py > gpurun_out/bg_c$c.log 2>&1 || exit $?
done
OCRK_GEMM_NT=1 OCRK_GEMM_NT_CFG=6 timeout -k 10 400 python -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -q -x -m gpu > gpurun_out/nt_tests.log 2>&1; echo "nt tests rc=$?"; tail -2 gpurun_out/nt_tests.log
