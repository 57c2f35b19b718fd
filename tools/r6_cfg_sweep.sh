#!/bin/bash
# NT tile configurations with the tap-uniform addressing (tools-only library, make exp):
# tools/bench_conv.py per configuration (fwd / dgrad / wgrad of every conv layer).
export OCRK_LIB=tools/libocrk_exp.so
set -o pipefail
out=gpurun_out/r6sw; mkdir -p $out
for c in -1 1 2 5 7 10 11 12 13 14 18; do
  OCRK_GEMM_NT_CFG=$c timeout -k 10 120 python3 -u tools/bench_conv.py > $out/c$c.log 2>&1 || { echo "cfg $c failed"; tail -3 $out/c$c.log; exit 1; }
  echo "== cfg $c"; grep -E "conv[4-8]|total" $out/c$c.log
done
