#!/bin/bash
# round 5, third GPU pass: fp32 training on the split (BPTT + weight gradients), its
# precision tests, an fp32 step trace and bench line, then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out/t_r5c
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_model.py -x -v -s -k "fp32 or precision_policy" --timeout 200 \
  --timeout-method thread > gpurun_out/t_r5c/policy.log 2>&1 || { tail -30 gpurun_out/t_r5c/policy.log; exit 1; }
grep -E "max relative|passed|failed" gpurun_out/t_r5c/policy.log | tail -4
timeout -k 10 200 python3 -u bench.py --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-cer > gpurun_out/t_r5c/fp32.json 2> gpurun_out/t_r5c/fp32.err || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/t_r5c/fp32.json
bash tools/quick_trace.sh r5fp32b --dtype fp32 || exit 1
bash tools/gpu_tests.sh r5c
