#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_trace.csv per (kernel, grid) -> avg/total time."""
import collections
import csv
import re
import sys


def summarise(path):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(list)
    for r in rows:
        m = re.search(r"::(k_\w+(?:<[^>]*>)?)\(", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        g = (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        agg[(name, g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = []
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        out.append(f"{k[0]:28s} grid={'x'.join(k[1]):18s} n={len(v):4d} "
                   f"avg={sum(v) / len(v) / 1e3:9.1f}us total={sum(v) / 1e6:8.2f}ms")
    return out


if __name__ == "__main__":
    print("\n".join(summarise(sys.argv[1])))
