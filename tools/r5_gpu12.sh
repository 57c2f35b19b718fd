#!/bin/bash
# conv row-kernel epilogue VALU trims: op parity, bf16 step parity, standalone conv timings, C3 A/B vs the previous library
set -o pipefail
mkdir -p gpurun_out/r5g12
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_bf16.py tests/test_gpu_bn_bf16.py tests/test_gpu_model.py > gpurun_out/r5g12/t.log 2>&1 || { tail -30 gpurun_out/r5g12/t.log; exit 1; }
tail -1 gpurun_out/r5g12/t.log
timeout -k 10 120 python3 tools/bench_conv.py > gpurun_out/r5g12/conv_new.txt 2>&1 || exit 1
OCRK_LIB=$PWD/tools/libocrk_prev.so timeout -k 10 120 python3 tools/bench_conv.py > gpurun_out/r5g12/conv_old.txt 2>&1 || exit 1
grep -E "^conv[2-5]" gpurun_out/r5g12/conv_old.txt gpurun_out/r5g12/conv_new.txt
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then L="OCRK_LIB=$PWD/tools/libocrk_prev.so"; else L=""; fi
    env $L timeout -k 10 150 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cer > gpurun_out/r5g12/${v}_$r.json 2>/dev/null || exit 1
  done
done
for v in new old; do echo "$v $(for f in gpurun_out/r5g12/${v}_*.json; do python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" $f; done | tr '\n' ' ')"; done
