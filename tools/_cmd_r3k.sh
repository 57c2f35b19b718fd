set -o pipefail
# conv NT tile sweep incl. deeper BK=32 pipelines, then the ping-pong-everywhere A/B
mkdir -p gpurun_out/r3k
for c in -1 2 5 11 12; do
  OCRK_GEMM_NT_CFG=$c timeout -k 10 120 python -u tools/bench_conv.py > gpurun_out/r3k/c$c.log 2>&1 || exit $?
  echo "cfg $c"; grep -v amdgpu.ids gpurun_out/r3k/c$c.log
done
OCRK_GEMM_PP=2 timeout -k 10 120 python -u tools/bench_conv.py > gpurun_out/r3k/pp2.log 2>&1 || exit $?
echo "pp2"; grep -v amdgpu.ids gpurun_out/r3k/pp2.log
