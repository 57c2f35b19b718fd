"""Per-launch HBM traffic of one kernel class from two rocprofv3 PMC passes.

    python tools/pmc_traffic.py --fetch DIR --write DIR --match SUBSTR --out FILE.json

FETCH_SIZE and WRITE_SIZE come from separate passes (they do not fit one TCC
pass on gfx950). Both are in KiB. MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so the
read side is doubled; WRITE_SIZE is exact for 16-B/lane stores.
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import re
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(root, counter, match, names=None):
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {root}")
    vals = defaultdict(float)
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter or not re.search(match, row.get("Kernel_Name", "")):
                    continue
                vals[(f, row.get("Dispatch_Id"))] += float(row["Counter_Value"])
                if names is not None:
                    names.add(row["Kernel_Name"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--match", required=True, help="regular expression on the kernel name")
    ap.add_argument("--desc", default="")
    ap.add_argument("--command", default="")
    ap.add_argument("--out", required=True)
    ap.add_argument("--lib", default=os.path.join(ROOT, "cnn_lstm_ctc_ocr_amd", "libocrk.so"),
                    help="the library the profiled run loaded: its sha256 ties the summary to the code "
                         "(bench.py reports the traffic only while the loaded library matches)")
    a = ap.parse_args()
    names = set()
    fetch = per_dispatch(a.fetch, "FETCH_SIZE", a.match, names)
    write = per_dispatch(a.write, "WRITE_SIZE", a.match)
    if not fetch or not write:
        raise SystemExit(f"no dispatches matching {a.match!r}")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    res = {
        "kernel_match": a.match,
        "kernel": a.desc,
        "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
        "fetch_size_kib_avg": round(f_kib, 2),
        "write_size_kib_avg": round(w_kib, 2),
        "read_bytes_per_launch": round(2 * f_kib * 1024),        # gfx950 FETCH_SIZE x2 correction
        "write_bytes_per_launch": round(w_kib * 1024),
        "bytes_per_launch": round((2 * f_kib + w_kib) * 1024),
        "command": a.command,
        "kernels": sorted(names),
        "libocrk_sha256": hashlib.sha256(open(a.lib, "rb").read()).hexdigest(),
    }
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
