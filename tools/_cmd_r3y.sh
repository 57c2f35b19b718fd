set -o pipefail
mkdir -p gpurun_out/r3y
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3y/gpu_tests.log 2>&1 || { tail -5 gpurun_out/r3y/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3y/gpu_tests.log
bash tools/evidence_round.sh r3y
