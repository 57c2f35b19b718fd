#!/bin/bash
# SQ counters of one GEMM shape (diagnostics): bash tools/pmc_gemm.sh tag "proj L2"
set -o pipefail
out=gpurun_out/pmc_gemm_${1:?tag}
mkdir -p "$out"
export TMPDIR=/tmp
cmd=(python3 tools/bench_gemm.py --only "${2:?shape}")
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $ctrs -d "$out/p$i" -o run --output-format csv -- "${cmd[@]}" \
        > "$out/p$i.log" 2>&1 || exit $?
done
python3 - "$out" <<'PY'
import csv, sys, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "gemm" not in n:
            continue
        agg[n.split("(")[0][-90:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.0f}")
PY
