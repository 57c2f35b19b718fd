#!/bin/bash
# SQ counters of the conv1 -> conv2 forward (tools/c12f_probe.py), GPU box, repo root.
set -o pipefail
out=gpurun_out/c12f; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/c12f_probe.py > $out/probe.txt 2>&1 || { tail -3 $out/probe.txt; exit 1; }
grep forward $out/probe.txt
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P3="SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH GRBM_COUNT"
i=0
for s in "$P1" "$P2" "$P3"; do
  timeout -s KILL 90 rocprofv3 --pmc $s -d "$out/p$i" -o run --output-format csv -- python3 tools/c12f_probe.py 5 \
      > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/p$i.log"; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py "$out/p0" "$out/p1" "$out/p2" > "$out/sq.txt" || exit 1
cat "$out/sq.txt"
