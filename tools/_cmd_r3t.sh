set -o pipefail
mkdir -p gpurun_out/r3t
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 250 --timeout-method thread -k "conv or bn or rows" > gpurun_out/r3t/tests.log 2>&1 || { tail -40 gpurun_out/r3t/tests.log; exit 1; }
tail -1 gpurun_out/r3t/tests.log
for v in 0 1; do echo "OCRK_CONV_ROWS_WIDE=$v"; OCRK_CONV_ROWS_WIDE=$v timeout -k 10 100 python -u tools/bench_conv.py 2>&1 | grep conv; done
for v in 0 1 0 1; do
  OCRK_CONV_ROWS_WIDE=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cer > gpurun_out/r3t/bench_$v.log 2>&1 || exit $?
  tail -1 gpurun_out/r3t/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('wide=$v', d['ms_per_step'], d['value'])"
done
