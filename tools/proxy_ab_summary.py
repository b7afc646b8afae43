#!/usr/bin/env python3
"""Means per configuration of a tools/proxy_ab.sh output file."""
import collections
import json
import sys

d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if " {" not in line:
        continue
    k, j = line.split(" {", 1)
    d[k].append(json.loads("{" + j)["ms_per_vcycle"])
for k, v in d.items():
    print(f"{k:28s} " + " ".join(f"{x:.4f}" for x in v) + f"  mean {sum(v) / len(v):.4f}")
