set -o pipefail
mkdir -p gpurun_out/r3n
for c in -1 2 3 5 11 12 13 14; do
  OCRK_GEMM_NT_CFG=$c timeout -k 10 60 python -u tools/bench_logits.py 2>&1 | grep cfg || exit 1
done
