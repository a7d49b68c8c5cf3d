"""Print a rocprofv3 --kernel-trace CSV as a timeline (ms from the first dispatch):
kernel, queue, start, duration, and which other kernels it overlapped.  Usage:
python tools/ktrace_timeline.py <kernel_trace.csv> [--from MS] [--to MS] [--match SUBSTR]"""
import argparse
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--from", dest="t0", type=float, default=0.0)
ap.add_argument("--to", dest="t1", type=float, default=1e12)
ap.add_argument("--match", default="")
args = ap.parse_args()
rows = list(csv.DictReader(open(args.csv)))
base = min(int(r["Start_Timestamp"]) for r in rows)
ks = []
for r in rows:
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("ik::", "").replace("vp8x::", "").replace("vp8::", "")
    s, e = (int(r["Start_Timestamp"]) - base) / 1e6, (int(r["End_Timestamp"]) - base) / 1e6
    ks.append((s, e, name, r["Queue_Id"], r["Grid_Size_X"]))
ks.sort()
for s, e, name, q, g in ks:
    if s < args.t0 or s > args.t1 or args.match not in name:
        continue
    ov = sorted({n for s2, e2, n, q2, _ in ks if n != name and s2 < e and e2 > s})
    print(f"{s:10.3f} {e - s:8.3f} q{q:>2} {name:28s} grid {g:>8s}  beside: {', '.join(ov)[:90]}")
