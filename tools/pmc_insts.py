"""Summarise an SQ-counter rocprofv3 pass (tools/pmc_insts.sh): per kernel, the counters summed over
its dispatches and divided by the dispatch count."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
files = glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in files:
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        short = name.split("(")[0].replace("void ", "")
        acc[short][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[short].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k in sorted(acc, key=lambda k: -acc[k].get("SQ_INSTS_VALU", 0)):
    n = max(1, len(disp[k]))
    c = {a: v / n for a, v in acc[k].items()}
    if c.get("SQ_INSTS_VALU", 0) < 1e6:
        continue
    print(f"{k}: dispatches {n}; per dispatch " + ", ".join(f"{a} {v:.4g}" for a, v in sorted(c.items())))
