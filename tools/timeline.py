"""One train step of a rocprofv3 kernel trace as a timeline: start/end
relative to the step start, stream, duration, kernel (short name). The step
is located by its Adam launch (the last kernel of a step)."""
import csv
import re
import sys


def short(n):
    n = n.replace("ocrk::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    return n[:70]


rows = list(csv.DictReader(open(sys.argv[1])))
step = int(sys.argv[2]) if len(sys.argv) > 2 else -2
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"].lower()]
lo = adam[step - 1] + 1
hi = adam[step] + 1
t0 = int(rows[lo]["Start_Timestamp"])
tot = int(rows[hi - 1]["End_Timestamp"]) - t0
print(f"# step span {tot / 1e3:.1f} us, {hi - lo} kernels")
for r in rows[lo:hi]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} q{r['Queue_Id']:>2} s{r['Stream_Id']:>2} {(e - s) / 1e3:7.1f} "
          f"g{r['Grid_Size_X']:>8} lds{r['LDS_Block_Size']:>6} {short(r['Kernel_Name'])}")
