#!/usr/bin/env python3
"""Turn one tools/profile.sh output directory into the committed summaries:

  profiles/<tag>_kernels.txt        per (kernel, grid) launch count / avg / total
                                    time from the rocprofv3 kernel trace
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats table, verbatim
  profiles/traffic_smoother.json    HBM bytes per launch of the smoother at the
                                    finest level (the bench's dominant kernel)

HBM bytes follow MI355X_MICROARCH.md "HBM [CDNA4]": on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read (x2), WRITE_SIZE
is exact for 16-B-per-lane stores; both are in KiB.

usage: make_profile_summary.py PROF_DIR TAG [--n 512 --world 1]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_summary import summarise  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    m = re.search(r"::(k_\w+(?:<[^>]*>)?)\(", name)
    return m.group(1) if m else name[:40]


def counters(path):
    """(kernel, grid) -> counter -> per-dispatch values, keeping only the
    longest-running cluster of dispatches (the finest MG level: the same
    kernel and grid can serve several levels)."""
    per = collections.defaultdict(list)
    for f in glob.glob(path):
        for r in csv.DictReader(open(f)):
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            per[(short(r["Kernel_Name"]), int(r["Grid_Size"]))].append(
                (dur, r["Counter_Name"], float(r["Counter_Value"])))
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for k, rows in per.items():
        top = max(d for d, _, _ in rows)
        for d, name, v in rows:
            if d >= top / 1.8:
                vals[k][name].append(v)
                vals[k]["_dur"].append(d)
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("tag")
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--kernel", default="k_gsrb")
    args = ap.parse_args()
    d = args.prof_dir
    trace = glob.glob(os.path.join(d, "trace", f"{args.tag}_kernel_trace.csv"))[0]
    stats = glob.glob(os.path.join(d, "trace", f"{args.tag}_kernel_stats.csv"))[0]
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", f"{args.tag}_kernels.txt"), "w") as f:
        f.write(f"# rocprofv3 --kernel-trace --stats -- python3 bench.py (tools/profile.sh), {args.tag}\n")
        f.write("\n".join(summarise(trace)) + "\n")
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{args.tag}_kernel_stats.csv"))

    fetch = counters(os.path.join(d, "pmc_fetch", f"{args.tag}_counter_collection.csv"))
    write = counters(os.path.join(d, "pmc_write", f"{args.tag}_counter_collection.csv"))
    # the dominant smoother launch: the (kernel, grid) with the most total
    # time in its finest-level cluster (the steady-state fine sweep)
    keys = [k for k in fetch if k[0].startswith(args.kernel)]
    if not keys:
        raise SystemExit("no smoother dispatches in the PMC passes")
    k = max(keys, key=lambda kk: sum(fetch[kk]["_dur"]))
    fb = sum(fetch[k]["FETCH_SIZE"]) / len(fetch[k]["FETCH_SIZE"]) * 1024 * 2
    wb = sum(write[k]["WRITE_SIZE"]) / len(write[k]["WRITE_SIZE"]) * 1024
    # the key bench.py looks up: colour passes per launch of that kernel
    kind = ("fused2x" if "tb2" in k[0] else
            "fused" if "fused" in k[0] or "block" in k[0] else "pass")
    out_path = os.path.join(ROOT, "profiles", "traffic_smoother.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    data[f"n{args.n}_w{args.world}_{kind}"] = {
        "kernel": k[0], "grid": k[1], "tag": args.tag,
        "read_bytes_per_launch": fb, "write_bytes_per_launch": wb,
        "hbm_bytes_per_launch": fb + wb,
        "launches_sampled": len(fetch[k]["FETCH_SIZE"]),
        "method": "FETCH_SIZE*1024*2 (gfx950 half-count correction) + WRITE_SIZE*1024, "
                  "separate --pmc passes",
    }
    json.dump(data, open(out_path, "w"), indent=1)
    print(json.dumps(data, indent=1))


if __name__ == "__main__":
    main()
