# A/B of the step under the engine / stream toggles (GPU box, repo root)
set -o pipefail
mkdir -p gpurun_out
for cfg in "OCRK_GEMM_NT=0 OCRK_SIDE_STREAM=0" "OCRK_GEMM_NT=1 OCRK_SIDE_STREAM=0" "OCRK_GEMM_NT=0 OCRK_SIDE_STREAM=1" "OCRK_GEMM_NT=1 OCRK_SIDE_STREAM=1"; do
  env $cfg timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit $?
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
done
