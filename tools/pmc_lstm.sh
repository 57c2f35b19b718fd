#!/bin/bash
# L2 hit rate and memory-side traffic of the recurrent step kernels (diagnostics).
# Run on the GPU box from the repo root:  bash tools/pmc_lstm.sh tag
set -o pipefail
out=gpurun_out/pmc_lstm_${1:?tag}
mkdir -p "$out"
export TMPDIR=/tmp
cmd=(python3 tools/bench_lstm.py 256)
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$out/hit" -o run --output-format csv -- "${cmd[@]}" \
    > "$out/hit.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- "${cmd[@]}" \
    > "$out/fetch.log" 2>&1 || exit $?
python3 - "$out" <<'PY'
import csv, sys, collections, glob
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "lstm" not in n:
            continue
        k = n.split("(")[0][-60:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    line = {c: sum(v) / len(v) for c, v in d.items()}
    hit = line.get("TCC_HIT_sum"); miss = line.get("TCC_MISS_sum")
    rate = hit / (hit + miss) if hit is not None and miss else None
    print(k, {c: round(v, 1) for c, v in line.items()}, "hit rate", rate)
PY
