#!/bin/bash
# SQ / LDS counter passes over one batched TN weight-gradient GEMM (tools/tn_one.py).
#   bash tools/pmc_tn.sh TAG M N
set -o pipefail
tag=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 60 python3 tools/tn_one.py "$@" 10 > "$out/time.txt" 2>&1 || exit $?
sets=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA"
      "GRBM_GUI_ACTIVE")
i=0
for s in "${sets[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $s -d "$out/p$i" -o run --output-format csv -- python3 tools/tn_one.py "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed: $s" >> "$out/failed.txt"; exit 1; }
  i=$((i+1))
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "pptn" not in r["Kernel_Name"] and "gemm" not in r["Kernel_Name"]:
            continue
        k = (r["Kernel_Name"][:60], r["Counter_Name"])
        tot[k] += float(r["Counter_Value"]); n[k] += 1
for (kn, c), v in sorted(tot.items()):
    print(f"{kn:60s} {c:28s} {v / max(n[(kn, c)], 1):16.1f}")
PY
