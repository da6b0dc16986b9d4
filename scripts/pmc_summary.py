"""Summarise rocprofv3 --pmc CSV passes per kernel: mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "?")
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    if "krr" not in k:
        continue
    print(k[:60])
    for c, v in sorted(cs.items()):
        # one row per dispatch (already summed over dimensions by rocprofv3 when it aggregates)
        print(f"   {c:28s} mean/dispatch {sum(v)/len(v):16.1f}   rows {len(v)}")
