"""Per-layer table of the conv1/conv2-conv8 forward launches of the bench step (conv1 -> conv2
as one launch, conv12_fwd_rows_kernel, when the bf16 step fuses them):
duration (rocprofv3 --kernel-trace), TFLOP/s and MFMA fraction, and HBM
bytes from the PMC passes (FETCH_SIZE x2 per the gfx950 correction +
WRITE_SIZE) against the algorithmic bytes (input + output activations +
weights, bf16). Dispatches are matched by kernel name and assigned to layers
in issue order (7 per step).

    python tools/conv_table.py --trace DIR --fetch DIR --write DIR --out FILE.md
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict

FWD = re.compile(r"conv3x3_direct_kernel<\d+, \d+, \d+, false|gemm_nt_kernel<(\d+, ){5}2, [48](, (false|true))*>|"
                 r"conv3x3_fwd_rows_kernel|conv3x3_fwd_rows_co_kernel|conv12_fwd_rows_kernel")
B = 256
LAYERS = [("conv2", 30, 254, 32, 32), ("conv3", 15, 127, 32, 64), ("conv4", 15, 127, 64, 64),
          ("conv5", 7, 126, 64, 128), ("conv6", 7, 126, 128, 128), ("conv7", 3, 125, 128, 256),
          ("conv8", 3, 125, 256, 256)]
PEAK = 2500.0   # dense bf16 TFLOP/s, MI355X_MICROARCH.md
HBM = 8.0       # TB/s, HBM3E spec


def rows(root, name):
    out = []
    for f in glob.glob(os.path.join(root, "**", name), recursive=True):
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


def short(n):
    n = n.replace("ocrk::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    tr = sorted((r for r in rows(a.trace, "*kernel_trace.csv") if FWD.search(r["Kernel_Name"])),
                key=lambda r: int(r["Start_Timestamp"]))
    dur = defaultdict(list)
    names = {}
    for i, r in enumerate(tr):
        layer = LAYERS[i % 7][0]
        dur[layer].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        names[layer] = short(r["Kernel_Name"])

    def pmc(root, counter):
        per = defaultdict(float)
        order = {}
        for r in rows(root, "*counter_collection.csv"):
            if r["Counter_Name"] == counter and FWD.search(r["Kernel_Name"]):
                key = int(r["Dispatch_Id"])
                per[key] += float(r["Counter_Value"])
                order[key] = int(r["Start_Timestamp"])
        keys = sorted(per, key=lambda k: order[k])
        out = defaultdict(list)
        for i, k in enumerate(keys):
            out[LAYERS[i % 7][0]].append(per[k] * 1024)
        return out

    fetch, write = pmc(a.fetch, "FETCH_SIZE"), pmc(a.write, "WRITE_SIZE")
    # each kernel against min(MFMA peak, AI x HBM bandwidth), AI = algorithmic
    # FLOP / algorithmic bytes (input + output activations + weights)
    lines = ["| layer | kernel | us | TFLOP/s | MFMA frac | AI FLOP/B | roofline TFLOP/s | roofline frac | "
             "algorithmic MB | counter MB | counter / algorithmic |",
             "|---|---|---|---|---|---|---|---|---|---|---|"]
    tot_us = tot_fl = 0.0
    for name, H, W, cin, cout in LAYERS:
        M = B * H * W
        fl = 2.0 * M * 9 * cin * cout
        alg = (M * cin + M * cout + 9 * cin * cout) * 2
        if name == "conv2" and "conv12" in names.get(name, ""):
            # conv1 -> conv2 in one launch: the u8 image in; y1 (bf16; not written by the
            # <XIN, false> form, whose backward recomputes it), its ReLU bit mask (4 B per
            # pixel) and z (bf16) out; both layers' weights
            fl = 2.0 * M * 9 * (1 * 32 + cin * cout)
            y1 = 0 if names[name].endswith("false>") else 2 * cin
            alg = B * (H + 2) * (W + 2) + M * (y1 + 4 + 2 * cout) + 9 * 32 * 4 + 9 * cin * cout * 2
            name_shown = "conv1+2 1->32->32"
        else:
            name_shown = f"{name} {cin}->{cout}"
        us = sum(dur[name]) / max(len(dur[name]), 1)
        rd = 2 * sum(fetch[name]) / max(len(fetch[name]), 1)
        wr = sum(write[name]) / max(len(write[name]), 1)
        tf = fl / us / 1e6
        ai = fl / alg
        roof = min(PEAK, ai * HBM)
        tot_us += us
        tot_fl += fl
        lines.append(f"| {name_shown} | `{names.get(name, '?')}` | {us:.1f} | {tf:.0f} | {tf / PEAK:.3f} | "
                     f"{ai:.0f} | {roof:.0f} | {tf / roof:.3f} | {alg / 1e6:.1f} | {(rd + wr) / 1e6:.1f} | "
                     f"{(rd + wr) / alg:.2f} |")
    tf = tot_fl / tot_us / 1e6
    lines.append(f"| all | | {tot_us:.1f} | {tf:.0f} | {tf / PEAK:.3f} | | | | | | |")
    txt = "\n".join(lines) + "\n"
    with open(a.out, "w") as fh:
        fh.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
