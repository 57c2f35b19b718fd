"""Per-kernel isolated duration and HBM bytes of one bench step from the two
PMC passes of tools/profile_round.sh (rocprofv3 serialises dispatches under
--pmc, so each duration is the kernel alone). Prints, per kernel name (summed
over its launches in the last profiled step), us, MB (FETCH_SIZE x2 + WRITE_SIZE,
gfx950 correction as in tools/pmc_traffic.py) and GB/s.

    python tools/kernel_bw.py gpurun_out/prof_r3a [--step-kernels 98]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def rows(root, counter):
    out = []
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == counter:
                    out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]),
                                int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out.sort()
    return out


def main():
    root = sys.argv[1]
    n = int(sys.argv[sys.argv.index("--step-kernels") + 1]) if "--step-kernels" in sys.argv else 0
    fe = rows(os.path.join(root, "fetch"), "FETCH_SIZE")
    wr = rows(os.path.join(root, "write"), "WRITE_SIZE")
    if n:
        fe, wr = fe[-n:], wr[-n:]
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for (d, name, f, s, e), (_, name2, w, _, _) in zip(fe, wr):
        short = name.replace("void ", "").replace("ocrk::(anonymous namespace)::", "").split("(")[0][:70]
        a = agg[short]
        a[0] += 1
        a[1] += (e - s) / 1e3
        a[2] += (2 * f + w) * 1024 / 1e6
    tot_us = sum(a[1] for a in agg.values())
    print(f"{'kernel':70s} {'n':>3s} {'us':>8s} {'MB':>8s} {'GB/s':>7s}")
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:70s} {a[0]:3d} {a[1]:8.1f} {a[2]:8.1f} {a[2] / max(a[1], 1e-9) * 1e3:7.0f}")
    print(f"total {tot_us:.1f} us")


if __name__ == "__main__":
    main()
