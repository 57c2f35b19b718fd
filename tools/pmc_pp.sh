#!/bin/bash
# PMC passes over one GEMM shape (tools/pp_one.py), one rocprofv3 run per counter set.
#   bash tools/pmc_pp.sh TAG M N K
set -o pipefail
tag=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
sets=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
      "TCC_HIT_sum TCC_MISS_sum"
      "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
      "GRBM_GUI_ACTIVE")
i=0
for s in "${sets[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $s -d "$out/p$i" -o run --output-format csv -- python3 tools/pp_one.py "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed: $s" >> "$out/failed.txt"; exit 1; }
  i=$((i+1))
done
true
