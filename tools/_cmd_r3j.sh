set -o pipefail
# A/B: ping-pong engine on every shape it covers (OCRK_GEMM_PP=2) vs the default routing
mkdir -p gpurun_out/r3j
for v in 1 2; do
  OCRK_GEMM_PP=$v timeout -k 10 120 python -u tools/bench_conv.py > gpurun_out/r3j/conv_pp$v.log 2>&1 || exit $?
  tail -1 gpurun_out/r3j/conv_pp$v.log
done
for v in 1 2 1 2; do
  OCRK_GEMM_PP=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cer > gpurun_out/r3j/bench_pp$v.log 2>&1 || exit $?
  tail -1 gpurun_out/r3j/bench_pp$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pp=$v', d['ms_per_step'], d['value'])"
done
