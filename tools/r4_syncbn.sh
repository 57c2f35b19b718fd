set -o pipefail
mkdir -p gpurun_out/syncbn
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_syncbn.py tests/test_gpu_dist.py tests/test_gpu_model.py -x -v --timeout 300 --timeout-method thread > gpurun_out/syncbn/tests.log 2>&1; rc=$?; tail -25 gpurun_out/syncbn/tests.log; exit $rc
