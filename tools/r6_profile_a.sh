#!/bin/bash
# (Historical: these runs used switches removed from the product in round 6 --
#  SIDE_CU_MASK, FORK_EVENTS, PP_DEEP, ... -- their results are kept under profiles/.)
# Round-6 counter passes (VERDICT r5 "next" #3, #4, #6), GPU box, repo root:
#  1. SQ counters of every conv forward / backward-data kernel of the bench
#     shape (tools/bench_conv.py): the NT engine on conv6-8 had none;
#  2. the ping-pong GEMM's L2 input projection (32000 x 4096 x 1024) with the
#     deep-lead schedule off and on (OCRK_PP_DEEP): did the wait fraction fall?
#  3. kernel-trace step timelines: default and the CU-masked side stream.
set -o pipefail
out=gpurun_out/r6pa
mkdir -p "$out"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum SQ_BUSY_CYCLES GRBM_COUNT"
i=0
for s in "$P1" "$P2" "$P3"; do
  timeout -s KILL 120 rocprofv3 --pmc $s -d "$out/conv$i" -o run --output-format csv -- python3 tools/bench_conv.py \
      > "$out/conv$i.log" 2>&1 || { echo "conv pass $i failed"; tail -5 "$out/conv$i.log"; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py "$out/conv0" "$out/conv1" "$out/conv2" > "$out/conv_sq.txt" || exit 1
for deep in 0 1; do
  i=0
  for s in "$P1" "$P2"; do
    OCRK_PP_DEEP=$deep timeout -s KILL 90 rocprofv3 --pmc $s -d "$out/pp${deep}_$i" -o run --output-format csv \
        -- python3 tools/pp_one.py 32000 4096 1024 > "$out/pp${deep}_$i.log" 2>&1 || { echo "pp pass failed"; exit 1; }
    i=$((i+1))
  done
  python3 tools/pmc_summary.py "$out/pp${deep}_0" "$out/pp${deep}_1" > "$out/pp_deep$deep.txt" || exit 1
done
bash tools/quick_trace.sh r6def || exit 1
OCRK_SIDE_CU_MASK=192 bash tools/quick_trace.sh r6mask192 || exit 1
cp gpurun_out/qt_r6def/step_timeline.txt "$out/step_timeline_default.txt"
cp gpurun_out/qt_r6mask192/step_timeline.txt "$out/step_timeline_mask192.txt"
cp gpurun_out/qt_r6def/kernel_stats.csv "$out/kernel_stats_default.csv"
echo done
