set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bnb
OCRK_BN_BWD_BLOCKS=512 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_syncbn.py tests/test_gpu_ops.py -k "bn or slab" -x -q --timeout 300 --timeout-method thread > gpurun_out/bnb/tests.log 2>&1; rc=$?; tail -2 gpurun_out/bnb/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh r4r || exit $?
bash tools/ab_env.sh bnb 3 "base:" "b1024:OCRK_BN_BWD_BLOCKS=1024" "b512:OCRK_BN_BWD_BLOCKS=512" || exit $?
