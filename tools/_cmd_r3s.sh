set -o pipefail
mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 250 --timeout-method thread -k "conv" > gpurun_out/r3s/tests.log 2>&1 || { tail -30 gpurun_out/r3s/tests.log; exit 1; }
tail -1 gpurun_out/r3s/tests.log
for v in 0 1; do echo "OCRK_CONV_ROWS=$v"; OCRK_CONV_ROWS=$v timeout -k 10 100 python -u tools/bench_conv.py 2>&1 | grep conv2; done
