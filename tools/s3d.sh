set -o pipefail
o=gpurun_out/s3d
mkdir -p $o
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit $?
timeout -k 10 100 python3 -u tools/bench_conv1.py > $o/conv1.log 2>&1 || exit $?
bash tools/ab_sched.sh > $o/ab.txt 2>&1 || exit $?
OCRK_TAIL=0 bash tools/quick_trace.sh s3d || exit $?
