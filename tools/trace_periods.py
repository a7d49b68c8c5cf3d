"""Stage periods from a rocprofv3 kernel trace of bench.py: the median gap between
successive launches of each key kernel (the steady-state step of the stage that
launches it) and the median durations.  Usage: python tools/trace_periods.py <kernel_trace.csv>"""
import csv
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
base = min(int(r["Start_Timestamp"]) for r in rows)
ks = {}
for r in rows:
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).split("::")[-1].split("<")[0]
    ks.setdefault(n, []).append(((int(r["Start_Timestamp"]) - base) / 1e6, (int(r["End_Timestamp"]) - base) / 1e6))
for n in ["k_png_wave", "k_png_find", "k_png_expand8", "k_png_resolve", "k_png_unfilter", "k_png_unfilter_su",
          "k_vp8x_run", "k_resize_fused", "k_png_gather"]:
    v = sorted(ks.get(n, []))
    if len(v) < 3:
        continue
    per = [v[i + 1][0] - v[i][0] for i in range(len(v) - 1)]
    per = [p for p in per if p < 80]  # the steady steps (not the legs between)
    dur = [e - s for s, e in v if e - s > 0.05]
    print(f"{n:18s} n={len(v):3d} period med {statistics.median(per) if per else 0:6.2f}  dur med {statistics.median(dur) if dur else 0:6.2f}")
w = sorted(ks.get("k_png_wave", []))
# the gap between the previous kernel on the decode stream ending and each wave starting
ends = sorted(e for n in ks for s, e in ks[n] if n.startswith("k_png_unfilter"))
gaps = []
for s, e in w:
    prev = [x for x in ends if x <= s]
    if prev and s - prev[-1] < 10:
        gaps.append(s - prev[-1])
if gaps:
    print(f"unfilter end -> wave start gap: median {statistics.median(gaps):.2f} ms over {len(gaps)}")
