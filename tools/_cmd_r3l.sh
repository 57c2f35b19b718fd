set -o pipefail
# bias reductions moved to the side stream: targeted GPU tests + A/B bench
mkdir -p gpurun_out/r3l
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_bf16.py tests/test_gpu_graph.py tests/test_gpu_persistent.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3l/tests.log 2>&1 || { tail -30 gpurun_out/r3l/tests.log; exit 1; }
tail -2 gpurun_out/r3l/tests.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cer > gpurun_out/r3l/bench_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/r3l/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'])"
done
