set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fork
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_images.py tests/test_gpu_graph.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fork/tests.log 2>&1; rc=$?; tail -5 gpurun_out/fork/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh fork2 3 "f1:" "f0:OCRK_FORK_EVENTS=0" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fork/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-cer > gpurun_out/fork/prof.log 2>&1 || exit $?
grep -h "copy_batch\|adam\|slab_sum" $(find gpurun_out/fork/prof -name '*kernel_stats.csv')
