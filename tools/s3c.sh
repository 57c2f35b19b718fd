# session-3 check: GPU tests, BN segment A/B, step A/B of stream toggles, one trace
set -o pipefail
o=gpurun_out/s3c
mkdir -p $o
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit $?
for sg in 1 2 4 8; do
  echo "OCRK_BN_SEG=$sg" >> $o/bn.log
  OCRK_BN_SEG=$sg timeout -k 10 100 python3 -u tools/bench_bn.py >> $o/bn.log 2>&1 || exit $?
done
bash tools/ab_sched.sh > $o/ab.txt 2>&1 || exit $?
bash tools/quick_trace.sh s3c || exit $?
