set -o pipefail
mkdir -p gpurun_out/r3q
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_model.py tests/test_gpu_bf16.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r3q/tests.log 2>&1 || { tail -30 gpurun_out/r3q/tests.log; exit 1; }
tail -1 gpurun_out/r3q/tests.log
for v in 0 1 0 1; do
  OCRK_PREFETCH_IMAGES=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cer > gpurun_out/r3q/bench_$v.log 2>&1 || exit $?
  tail -1 gpurun_out/r3q/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('prefetch=$v', d['ms_per_step'], d['value'])"
done
