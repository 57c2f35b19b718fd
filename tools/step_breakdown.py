"""Per-train-step kernel time breakdown from a rocprofv3 kernel trace (diagnostics).

    python tools/step_breakdown.py gpurun_out/prof_r1d/trace/run_kernel_trace.csv [--top 30]

A step is the span between two consecutive Adam launches (the last kernel of
a train step). Times are summed busy time per kernel family over the last
complete step, split by HIP stream (main vs side); the wall span of the step
is printed too, so overlap shows as sum(busy) > wall.
"""
import argparse
import collections
import csv
import re


def family(name):
    n = name.split("(")[0]
    n = re.sub(r"^void ", "", n)
    m = re.match(r"_Z\d+(\w+?)I", n)
    if m:
        n = m.group(1)
    n = re.sub(r"<.*", "", n)
    # keep the tile config of the GEMM engines: it tells the call sites apart
    t = re.search(r"gemm_(nt|tn)_kernel<([^>]*)>", name)
    if t:
        n = f"gemm_{t.group(1)}<{t.group(2)}>"
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"].lower()]
    # the Adam launches of one step are contiguous: step boundary = last of a run
    last = [i for k, i in enumerate(ends) if k + 1 == len(ends) or ends[k + 1] != i + 1]
    if len(last) < 2:
        raise SystemExit("need two complete steps in the trace")
    lo, hi = last[-2] + 1, last[-1] + 1
    step = rows[lo:hi]
    wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    busy = collections.defaultdict(float)
    cnt = collections.Counter()
    by_stream = collections.defaultdict(float)
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        f = family(r["Kernel_Name"])
        busy[f] += d
        cnt[f] += 1
        by_stream[r.get("Stream_Id", "?")] += d
    tot = sum(busy.values())
    print(f"step wall {wall / 1e3:.3f} ms, kernel busy {tot / 1e3:.3f} ms, {len(step)} launches")
    for s, v in sorted(by_stream.items()):
        print(f"  stream {s}: {v / 1e3:.3f} ms busy")
    for f, v in sorted(busy.items(), key=lambda kv: -kv[1])[: a.top]:
        print(f"{v / 1e3:8.3f} ms {cnt[f]:5d}x {v / cnt[f]:9.2f} us  {f}")


if __name__ == "__main__":
    main()
