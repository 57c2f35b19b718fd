set -o pipefail
# (Historical: these runs used switches removed from the product in round 6 --
#  SIDE_CU_MASK, FORK_EVENTS, PP_DEEP, ... -- their results are kept under profiles/.)
mkdir -p gpurun_out/syncbn
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_syncbn.py tests/test_gpu_images.py tests/test_gpu_ops.py tests/test_gpu_dist.py tests/test_gpu_model.py -x -v --timeout 300 --timeout-method thread > gpurun_out/syncbn/tests.log 2>&1; rc=$?; tail -25 gpurun_out/syncbn/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/syncbn/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-cer > gpurun_out/syncbn/prof.log 2>&1 || exit $?
grep -h "copy_batch\|adam\|slab_sum" $(find gpurun_out/syncbn/prof -name '*kernel_stats.csv')
grep '^{' gpurun_out/syncbn/prof.log | tail -1 | cut -c1-300
bash tools/ab_env.sh fork 3 "base:" "f1:OCRK_FORK_EVENTS=1" "f2:OCRK_FORK_EVENTS=2"
