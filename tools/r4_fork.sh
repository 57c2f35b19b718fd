set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fork
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_images.py tests/test_gpu_graph.py tests/test_gpu_syncbn.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fork/tests.log 2>&1; rc=$?; tail -5 gpurun_out/fork/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh r4o || exit $?
grep -h "copy_batch\|adam\|slab_sum" gpurun_out/prof_r4o/kernel_stats.csv
bash tools/ab_env.sh fork2 2 "f1:" "f0:OCRK_FORK_EVENTS=0" || exit $?
