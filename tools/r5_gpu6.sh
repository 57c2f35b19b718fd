#!/bin/bash
# fp32 persistent BPTT: parity tests, the fp32 model/trainer tests, fp32 bench + kernel stats
set -o pipefail
mkdir -p gpurun_out/r5g6
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_persistent.py -k "f32" > gpurun_out/r5g6/t_pers.log 2>&1 || { tail -40 gpurun_out/r5g6/t_pers.log; exit 1; }
grep -E "rel err|passed|failed" gpurun_out/r5g6/t_pers.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread \
  tests/test_gpu_model.py tests/test_gpu_configs.py -k "fp32 or f32" > gpurun_out/r5g6/t_model.log 2>&1 || { tail -40 gpurun_out/r5g6/t_model.log; exit 1; }
tail -3 gpurun_out/r5g6/t_model.log
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline --breakdown > gpurun_out/r5g6/bench_fp32.json 2> gpurun_out/r5g6/bench_fp32.err || { tail -20 gpurun_out/r5g6/bench_fp32.err; exit 1; }
cat gpurun_out/r5g6/bench_fp32.json
