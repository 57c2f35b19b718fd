set -o pipefail
# (Historical: these runs used switches removed from the product in round 6 --
#  SIDE_CU_MASK, FORK_EVENTS, PP_DEEP, ... -- their results are kept under profiles/.)
export TMPDIR=/tmp
mkdir -p gpurun_out/fork3
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_images.py tests/test_gpu_graph.py tests/test_gpu_model.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fork3/tests.log 2>&1; rc=$?; tail -3 gpurun_out/fork3/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh fork3 4 "f1:" "f0:OCRK_FORK_EVENTS=0" || exit $?
bash tools/profile_round.sh r4p || exit $?
grep -h "copy_batch\|adam\|slab_sum" gpurun_out/prof_r4p/kernel_stats.csv
