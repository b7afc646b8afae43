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
    # one (kernel, grid) can serve several MG levels (the streaming sweep
    # launches one workgroup per CU slot at every level): split by duration
    rows = []
    for k, v in agg.items():
        for c in clusters(v):
            rows.append((k, c))
    out = []
    for k, v in sorted(rows, key=lambda kv: -sum(kv[1])):
        out.append(f"{k[0]:28s} grid={'x'.join(k[1]):18s} n={len(v):4d} "
                   f"avg={sum(v) / len(v) / 1e3:9.1f}us total={sum(v) / 1e6:8.2f}ms")
    return out


def timeline(path, last=90):
    """The last `last` launches in start order: duration and idle gap before."""
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out, prev = [], None
    for r in rows[-last:]:
        m = re.search(r"::(k_\w+(?:<[^>]*>)?)\(", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        prev = e
        g = "x".join((r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"]))
        out.append(f"{name[:60]:60s} grid={g:16s} dur={(e - s) / 1e3:9.1f}us gap={gap:8.1f}us")
    return out


def clusters(durations, gap=1.8):
    """Split durations into groups separated by a jump of more than `gap`x."""
    v = sorted(durations)
    out, cur = [], [v[0]]
    for d in v[1:]:
        if d > gap * cur[-1]:
            out.append(cur)
            cur = [d]
        else:
            cur.append(d)
    out.append(cur)
    return out


if __name__ == "__main__":
    print("\n".join(summarise(sys.argv[1])))
    print("--- last launches (start order) ---")
    print("\n".join(timeline(sys.argv[1])))
