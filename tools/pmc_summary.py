#!/usr/bin/env python3
"""Average rocprofv3 counter values per kernel over the dispatches in one or
more *_counter_collection.csv files."""
import collections
import csv
import glob
import re
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for f in glob.glob(path):
        for r in csv.DictReader(open(f)):
            m = re.search(r"::(k_\w+(?:<[^>]*>)?)\(", r["Kernel_Name"])
            name = (m.group(1) if m else r["Kernel_Name"][:40]) + f" grid={r.get('Grid_Size', '')}"
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} n={len(v):4d} avg={sum(v) / len(v):.4e}")
