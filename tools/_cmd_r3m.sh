set -o pipefail
mkdir -p gpurun_out/r3m
for v in 0 1 0 1 0 1; do
  OCRK_DEFER_BIAS=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cer > gpurun_out/r3m/bench_$v.log 2>&1 || exit $?
  tail -1 gpurun_out/r3m/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('defer=$v', d['ms_per_step'], d['value'])"
done
