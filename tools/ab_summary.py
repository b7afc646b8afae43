#!/usr/bin/env python3
"""Summary of an A/B file written by the round-5 session scripts: per
variant the bench_smoother launch times (512^3 / 256^3, ms by events), the
bench.py V-cycles/s and frac of each interleaved round, and the checksums
(which must be one value per size).  usage: ab_summary.py FILE"""
import collections
import json
import sys

d = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(sys.argv[1]):
    j = json.loads(line)
    v = j["variant"]
    if "n" in j:
        d[v]["n%d" % j["n"]].append(j["ms_per_launch_events"])
        d[v]["ck%d" % j["n"]].append(j["checksum"])
    else:
        d[v]["vc"].append(j["vcycles"])
        d[v]["fr"].append(j["frac"])
for v, x in d.items():
    def avg(k):
        return sum(x[k]) / len(x[k]) if x[k] else float("nan")
    print(f"{v:8s} 512: {x['n512']} (avg {avg('n512'):.4f})  256: {x['n256']} (avg {avg('n256'):.4f})  "
          f"V-cycles/s {x['vc']} (avg {avg('vc'):.2f})  frac {x['fr']}  checksums "
          f"{sorted(set(x['ck512']))} {sorted(set(x['ck256']))}")
