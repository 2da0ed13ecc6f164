"""Summarise rocprofv3 PMC passes per kernel (mean over dispatches)."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?")
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
dur = defaultdict(list)
for f in glob.glob(os.path.join(root, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        dur[row["Name"]] = float(row["AverageNs"])
for k, d in vals.items():
    if "tokenize" not in k and "lane" not in k and "compact" not in k and "finish" not in k:
        continue
    short = k.split("(")[0][-60:]
    print(short, " avg_ns=%s" % next((v for n, v in dur.items() if n.split("(")[0] == k.split("(")[0]), "?"))
    for c, v in sorted(d.items()):
        print("   %-32s %16.4g" % (c, sum(v) / len(v)))
