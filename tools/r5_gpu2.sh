#!/bin/bash
# round 5, second GPU pass: trained-weight parity, fp32 precision policies, CU-limited side
# stream A/B, an fp32 step trace, the whole GPU suite
set -o pipefail
mkdir -p gpurun_out/t_r5b
OCRK_CURVES_OUT=gpurun_out/trained_r5b.json timeout -k 10 600 python3 -u -m pytest tests/test_gpu_trained.py -x -v -s \
  --timeout 400 --timeout-method thread > gpurun_out/t_r5b/trained.log 2>&1 || { tail -30 gpurun_out/t_r5b/trained.log; exit 1; }
grep -E "trained-weight|CER|windows" gpurun_out/t_r5b/trained.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py -x -v -s -k "precision_policy or fp32" --timeout 200 \
  --timeout-method thread > gpurun_out/t_r5b/policy.log 2>&1; grep -E "max relative|passed|failed|Error" gpurun_out/t_r5b/policy.log | tail -8
bash tools/ab_env.sh r5cu 2 "base:" "m224:OCRK_SIDE_CU_MASK=224" "m192:OCRK_SIDE_CU_MASK=192" || exit 1
bash tools/quick_trace.sh r5fp32 --dtype fp32 || exit 1
bash tools/gpu_tests.sh r5b
