set -o pipefail
mkdir -p gpurun_out/r3u
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3u/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3u/gpu_tests.log
exit $rc
