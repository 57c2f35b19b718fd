set -o pipefail
mkdir -p gpurun_out/r3r
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bn_bf16.py -x -q --timeout 250 --timeout-method thread -k "bn or deferred" > gpurun_out/r3r/tests.log 2>&1 || { tail -30 gpurun_out/r3r/tests.log; exit 1; }
tail -1 gpurun_out/r3r/tests.log
for v in 0 1; do echo "OCRK_BN_COL=$v"; OCRK_BN_COL=$v timeout -k 10 100 python -u tools/bench_bn.py 2>&1 | grep conv; done
