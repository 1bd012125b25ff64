"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (mean per dispatch)."""
import collections
import csv
import glob
import os
import sys

root, cfg = sys.argv[1], sys.argv[2]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, f"{cfg}_*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0][-40:]
        per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in per.items():
    if not k.strip().startswith("void nsd") and "nsd::" not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}")
