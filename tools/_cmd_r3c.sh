set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 120 python -u tools/bench_persist.py > gpurun_out/r3c/persist.txt 2>&1 || { cat gpurun_out/r3c/persist.txt; exit 1; }
for late in 0 1; do
  OCRK_PERSIST_LATE=$late timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cer > gpurun_out/r3c/bench_late$late.log 2>&1 || exit $?
done
cat gpurun_out/r3c/persist.txt
for late in 0 1; do tail -1 gpurun_out/r3c/bench_late$late.log | cut -c1-200; done
