"""Per-kernel summary of rocprofv3 --pmc passes: every *counter_collection.csv
under the given directories, libocrk kernels only, grouped by (kernel name,
grid size) -- the grid tells the conv layers apart -- and averaged per
dispatch. Prints the counters (millions) plus the ratios the SQ counters give
directly: WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY as fractions of
WAVE_CYCLES (disjoint; the guide's PMC section), LDS bank conflicts per LDS
cycle, VALU instructions per MFMA-busy kilocycle, the kernel's duration.

    python tools/pmc_summary.py DIR [DIR ...] [--match SUBSTR]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(n):
    n = n.replace("ocrk::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)[:90]


def main(argv):
    match = None
    if "--match" in argv:
        i = argv.index("--match")
        match = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    vals = defaultdict(lambda: defaultdict(list))     # key -> counter -> [per-dispatch]
    dur = defaultdict(dict)
    for d in argv:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            meta = {}
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if "ocrk" not in name or (match and match not in name):
                    continue
                k = (short(name), int(r["Grid_Size"]), r["Dispatch_Id"])
                per[(k, r["Counter_Name"])] += float(r["Counter_Value"])
                meta[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            for (k, c), v in per.items():
                vals[k[:2]][c].append(v)
                dur[k[:2]][k[2]] = meta[k]
    for key in sorted(vals, key=lambda k: -sum(dur[k].values())):
        cs = vals[key]
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        us = sum(dur[key].values()) / max(1, len(dur[key]))
        out = [f"{key[0]} grid={key[1]} dispatches={len(dur[key])} avg {us:.1f} us"]
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in avg:
                    out.append(f"  {c}/WAVE_CYCLES = {avg[c] / wc:.3f}")
        if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE"):
            out.append(f"  LDS_BANK_CONFLICT/LDS_IDX_ACTIVE = {avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "SQ_INSTS_VALU" in avg and avg.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            out.append(f"  VALU insts per MFMA-busy kcycle = {avg['SQ_INSTS_VALU'] / avg['SQ_VALU_MFMA_BUSY_CYCLES'] * 1e3:.1f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg and avg["GRBM_GUI_ACTIVE"]:
            # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles; MFMA busy summed over the 1024 SIMDs
            out.append(f"  MFMA busy / (GUI_ACTIVE/8 x 1024 SIMDs) = "
                       f"{avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
        out.append("  " + ", ".join(f"{c}={v / 1e6:.3f}M" for c, v in sorted(avg.items())))
        print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1:])
