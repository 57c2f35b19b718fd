set -o pipefail
mkdir -p gpurun_out/r3h
for v in 0 1 0 1; do
  OCRK_DEFER_DWX=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cer > gpurun_out/r3h/bench_$v.log 2>&1 || exit $?
  echo "defer=$v $(tail -1 gpurun_out/r3h/bench_$v.log | cut -c90-150)"
done
