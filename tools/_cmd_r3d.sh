set -o pipefail
mkdir -p gpurun_out/r3d
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3d/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3d/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3d/gpu_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3d/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-cer > gpurun_out/r3d/trace.log 2>&1 || exit $?
python3 tools/timeline.py "$(find gpurun_out/r3d/trace -name '*kernel_trace.csv' | head -1)" > gpurun_out/r3d/timeline.txt || exit $?
find gpurun_out/r3d/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/r3d/kernel_stats.csv \;
head -3 gpurun_out/r3d/timeline.txt
