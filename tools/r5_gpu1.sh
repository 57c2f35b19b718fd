#!/bin/bash
# round 5, first GPU pass: the deep-lead GEMM schedule (parity, then A/B), trained-weight
# parity, a CU-limited side stream A/B, an fp32 step trace, the whole GPU suite
set -o pipefail
mkdir -p gpurun_out/t_r5a
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bf16.py -x -v -k "pp_deep or plain_gemms" --timeout 120 \
  --timeout-method thread > gpurun_out/t_r5a/deep.log 2>&1 || { tail -30 gpurun_out/t_r5a/deep.log; exit 1; }
tail -2 gpurun_out/t_r5a/deep.log
bash tools/r5_pp_ab.sh > /dev/null || exit 1
grep -E "==|proj|dx" gpurun_out/pp/ab.txt
OCRK_CURVES_OUT=gpurun_out/trained_r5a.json timeout -k 10 600 python3 -u -m pytest tests/test_gpu_trained.py -x -v -s \
  --timeout 400 --timeout-method thread > gpurun_out/t_r5a/trained.log 2>&1 || { tail -30 gpurun_out/t_r5a/trained.log; exit 1; }
grep -E "trained-weight|CER|windows" gpurun_out/t_r5a/trained.log
bash tools/ab_env.sh r5cu 2 "base:" "deep:OCRK_PP_DEEP=1" "m224:OCRK_SIDE_CU_MASK=224" "m192:OCRK_SIDE_CU_MASK=192" || exit 1
bash tools/quick_trace.sh r5fp32 --dtype fp32 || exit 1
bash tools/gpu_tests.sh r5a
