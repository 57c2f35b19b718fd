"""Per-kernel-class table of one bench step from a rocprofv3 kernel trace and
(optionally) the FETCH_SIZE / WRITE_SIZE PMC passes of the same command: per
class the launches and time per step, and -- where PMC files are given -- the
counter HBM bytes per step and the achieved HBM bandwidth as a fraction of the
8 TB/s roofline (the bound of the BN, pool, reduce and copy kernels, which do
no MFMA work). Counter bytes = 2 x FETCH_SIZE + WRITE_SIZE (the
gfx950 read correction, MI355X_MICROARCH.md). Kernel time on a side stream
includes the time its workgroups share the CUs with the main stream's.

    python tools/kernel_table.py --trace DIR [--fetch DIR --write DIR] --steps N --out FILE.md
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict

HBM = 8000.0    # GB/s


def rows(root, name):
    out = []
    for f in glob.glob(os.path.join(root, "**", name), recursive=True):
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


def short(n):
    n = n.replace("ocrk::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    return n[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--steps", type=int, required=True, help="steps the trace covers (warm-up + timed)")
    ap.add_argument("--pmc-steps", type=int, default=None, help="steps the PMC runs cover")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    t = defaultdict(float)
    n = defaultdict(int)
    for r in rows(a.trace, "*kernel_trace.csv"):
        k = short(r["Kernel_Name"])
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        n[k] += 1
    byts = defaultdict(float)
    if a.fetch and a.write:
        for root, counter, mul in ((a.fetch, "FETCH_SIZE", 2.0), (a.write, "WRITE_SIZE", 1.0)):
            for r in rows(root, "*counter_collection.csv"):
                if r["Counter_Name"] == counter:
                    byts[short(r["Kernel_Name"])] += mul * float(r["Counter_Value"]) * 1024
    ps = a.pmc_steps or a.steps
    tot = sum(t.values()) / a.steps
    lines = [f"# kernel time per step {tot:.1f} us (sum over streams), {a.steps} steps traced", "",
             "| kernel | launches/step | us/step | share | counter MB/step | GB/s | HBM roofline frac |",
             "|---|---|---|---|---|---|---|"]
    for k in sorted(t, key=lambda k: -t[k]):
        us = t[k] / a.steps
        mb = byts[k] / ps / 1e6 if k in byts else None
        gbs = mb * 1e3 / us if mb else None
        lines.append(f"| `{k}` | {n[k] / a.steps:.1f} | {us:.1f} | {us / tot:.3f} | "
                     f"{'' if mb is None else f'{mb:.1f}'} | {'' if gbs is None else f'{gbs:.0f}'} | "
                     f"{'' if gbs is None else f'{gbs / HBM:.3f}'} |")
    txt = "\n".join(lines) + "\n"
    with open(a.out, "w") as fh:
        fh.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
