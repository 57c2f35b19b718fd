set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_gru
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gru/trace -o run --output-format csv -- python3 bench.py --cell gru --steps 5 --warmup 2 --no-cpu-baseline --no-cer > gpurun_out/prof_gru/trace.log 2>&1 || exit $?
find gpurun_out/prof_gru/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_gru/kernel_stats.csv \;
python3 tools/timeline.py "$(find gpurun_out/prof_gru/trace -name '*kernel_trace.csv' | head -1)" > gpurun_out/prof_gru/step_timeline.txt
head -3 gpurun_out/prof_gru/step_timeline.txt
