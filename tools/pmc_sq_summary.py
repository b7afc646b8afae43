"""Per-kernel means of SQ / GRBM counters from rocprofv3 --pmc passes
(tools/r04_session_pmc_sq.sh): every *_counter_collection.csv under the
given directory, grouped by (kernel, grid size), one mean per counter per
dispatch, plus the shares of SQ_WAVE_CYCLES (wait / issue-stall / active);
PMC_KERNELS: a regex of the kernels shown (default tb2).
Measurement tooling only."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main(d):
    per = defaultdict(lambda: defaultdict(dict))  # (kernel, grid) -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+(?:<[^()]*>)?)", r["Kernel_Name"])
            k = (m.group(1) if m else r["Kernel_Name"][:60], int(r["Grid_Size"]))
            key = (os.path.dirname(f), r.get("Dispatch_Id", ""))
            per[k][r["Counter_Name"]][key] = per[k][r["Counter_Name"]].get(key, 0.0) + float(r["Counter_Value"])
    for k, cs in sorted(per.items(), key=lambda kv: -len(next(iter(kv[1].values())))):
        if not re.search(os.environ.get("PMC_KERNELS", "tb2"), k[0]):
            continue
        print(f"{k[0]} grid={k[1]}")
        mean = {c: sum(v.values()) / len(v) for c, v in cs.items()}
        for c in sorted(mean):
            print(f"  {c:28s} {mean[c]:16.1f}  (n={len(cs[c])})")
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA"):
                if c in mean:
                    print(f"  share {c:22s} {mean[c] / wc:6.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
