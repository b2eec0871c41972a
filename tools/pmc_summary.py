#!/usr/bin/env python3
"""Sum rocprofv3 counter_collection CSVs per kernel name (mean per dispatch)."""
import collections
import csv
import glob
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0][-40:]
        rows[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in rows.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v) / len(v):16.1f}  (n={len(v)})")
