"""Dev tool: average each PMC counter per dispatch of a kernel (name substring) over
rocprofv3 --pmc CSV outputs.  Usage: python tools/pmc_summary.py KERNEL dir1 [dir2 ...]"""
import collections, csv, sys
kn = sys.argv[1]
for d in sys.argv[2:]:
    agg = collections.defaultdict(float); n = collections.Counter(); dur = []
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if kn not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(d, f"avg dispatch {sum(dur)/max(len(dur),1):.1f} us")
    for k in sorted(agg):
        print(f"  {k:28s} {agg[k]/n[k]:16.0f}")
