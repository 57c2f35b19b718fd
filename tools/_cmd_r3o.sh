set -o pipefail
mkdir -p gpurun_out/r3o
timeout -k 10 300 python -u -m pytest tests/test_gpu_ctc.py tests/test_gpu_golden.py tests/test_gpu_model.py tests/test_gpu_configs.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r3o/tests.log 2>&1 || { tail -30 gpurun_out/r3o/tests.log; exit 1; }
tail -1 gpurun_out/r3o/tests.log
timeout -k 10 60 python -u tools/bench_ctc.py 2>&1 | grep OCRK
timeout -k 10 60 python -u tools/bench_ctc.py --long 2>&1 | grep OCRK
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cer > gpurun_out/r3o/bench_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/r3o/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'])"
done
