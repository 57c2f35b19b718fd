set -o pipefail
mkdir -p gpurun_out/r3g
export TMPDIR=/tmp
for c in c2 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g/trace_$c -o run --output-format csv -- python3 bench.py --config $c --steps 8 --warmup 2 > gpurun_out/r3g/trace_$c.log 2>&1 || exit $?
  find gpurun_out/r3g/trace_$c -name "*kernel_stats.csv" -exec cp {} gpurun_out/r3g/kernel_stats_$c.csv \;
  tail -1 gpurun_out/r3g/trace_$c.log | cut -c1-250
done
