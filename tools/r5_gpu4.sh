#!/bin/bash
# round 5, fourth GPU pass: exact-mode fp32 convolutions on the NT ring, the fp32 step
# (both precision policies), a bf16 default bench line, the whole GPU suite
set -o pipefail
mkdir -p gpurun_out/t_r5d
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -v -s \
  -k "f32_exact_conv or precision_policy or fp32" --timeout 200 --timeout-method thread \
  > gpurun_out/t_r5d/f32.log 2>&1 || { tail -30 gpurun_out/t_r5d/f32.log; exit 1; }
grep -E "max relative|passed|failed" gpurun_out/t_r5d/f32.log | tail -4
for cfg in "mixed:" "mixed_generic:OCRK_NT_F32_EXACT=0" "exact:OCRK_F32_TRAIN_EXACT=1"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python3 -u bench.py --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-cer \
    > gpurun_out/t_r5d/fp32_$name.json 2> gpurun_out/t_r5d/fp32_$name.err || exit 1
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/t_r5d/fp32_$name.json)"
done
bash tools/quick_trace.sh r5fp32c --dtype fp32 || exit 1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-cer > gpurun_out/t_r5d/bf16.json 2> gpurun_out/t_r5d/bf16.err || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/t_r5d/bf16.json
bash tools/gpu_tests.sh r5d
