#!/bin/bash
# SQ stall breakdown of the per-layer conv kernels (tools/bench_conv.py), one
# rocprofv3 --pmc pass (8 SQ counters), for profiles/.
set -o pipefail
out=gpurun_out/pmc_sq
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -d "$out/sq" -o run --output-format csv \
    -- python3 tools/bench_conv.py > "$out/sq.log" 2>&1
