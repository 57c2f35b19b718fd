#!/bin/bash
# SQ counters + HBM bytes of the conv row kernels (tools/bench_conv.py), two --pmc passes
set -o pipefail
out=gpurun_out/pmc_rows; mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -d "$out/sq" -o run --output-format csv \
    -- python3 tools/bench_conv.py > "$out/sq.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d "$out/sq2" -o run --output-format csv \
    -- python3 tools/bench_conv.py > "$out/sq2.log" 2>&1 || exit 1
tail -12 "$out/sq.log"
