set -o pipefail
mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 250 --timeout-method thread -k "conv or bn" > gpurun_out/r3s/tests.log 2>&1 || { tail -30 gpurun_out/r3s/tests.log; exit 1; }
tail -1 gpurun_out/r3s/tests.log
for v in 0 1; do echo "OCRK_CONV_ROWS=$v"; OCRK_CONV_ROWS=$v timeout -k 10 100 python -u tools/bench_conv.py 2>&1 | grep conv; done
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bf16.py tests/test_gpu_graph.py tests/test_gpu_golden.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r3s/tests2.log 2>&1 || { tail -30 gpurun_out/r3s/tests2.log; exit 1; }
tail -1 gpurun_out/r3s/tests2.log
for v in 0 1 0 1; do
  OCRK_CONV_ROWS=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cer > gpurun_out/r3s/bench_$v.log 2>&1 || exit $?
  tail -1 gpurun_out/r3s/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rows=$v', d['ms_per_step'], d['value'])"
done
