set -o pipefail
mkdir -p gpurun_out/r3f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3f/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3f/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3f/gpu_tests.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cer > gpurun_out/r3f/bench.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --cell gru --no-cpu-baseline > gpurun_out/r3f/bench_gru.log 2>&1 || exit $?
tail -1 gpurun_out/r3f/bench.log | cut -c1-200; tail -1 gpurun_out/r3f/bench_gru.log | cut -c1-200
