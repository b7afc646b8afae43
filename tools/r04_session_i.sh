#!/bin/bash
# round-4 GPU session i: exchange block size x grid cap x loads in flight per
# thread (u8 = 8 instead of 4) on the 8-GPU share proxy.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/proxy_ab.txt
CONFIGS="new:2048:0 new:1024:0 new:2048:512 new:1024:512 new:4096:0 u8:4096:0 u8:2048:0 u8:2048:512 new:1024:1024" ROUNDS=2 bash tools/proxy_ab.sh || exit 1
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for line in open("gpurun_out/proxy_ab.txt"):
    k, j = line.split(" {", 1)
    d[k].append(json.loads("{" + j)["ms_per_vcycle"])
for k, v in d.items():
    print(f"{k:28s} " + " ".join(f"{x:.4f}" for x in v) + f"  mean {sum(v)/len(v):.4f}")
PY
echo "session done"
