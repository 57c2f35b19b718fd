set -o pipefail
mkdir -p gpurun_out/r3b
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/bench_persist.py > gpurun_out/r3b/persist.txt 2>&1 || exit $?
for f in 1 0; do
  OCRK_LSTM_BWD_KSPLIT=$f timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3b/trace_$f -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-cer > gpurun_out/r3b/trace_$f.log 2>&1 || exit $?
  python3 tools/timeline.py "$(find gpurun_out/r3b/trace_$f -name '*kernel_trace.csv' | head -1)" > gpurun_out/r3b/timeline_$f.txt || exit $?
done
cat gpurun_out/r3b/persist.txt
