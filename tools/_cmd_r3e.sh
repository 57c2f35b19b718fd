set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_gpu_gru_persistent.py tests/test_gpu_persistent.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3e/tests.log 2>&1 || { tail -30 gpurun_out/r3e/tests.log; exit 1; }
tail -1 gpurun_out/r3e/tests.log
timeout -k 10 200 python -u bench.py --cell gru --no-cpu-baseline > gpurun_out/r3e/bench_gru.log 2>&1 || exit $?
tail -1 gpurun_out/r3e/bench_gru.log | cut -c1-220
