#!/bin/bash
# rocprofv3 kernel trace of the whole-split proxy (tools/rank_proxy.py --parts
# 2,2,2 --size 512, agglomerated coarsest depth) -> gpurun_out/ts_split.txt.
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ts" -o ts --output-format csv -- python3 "$R/tools/rank_proxy.py" --size 512 --parts 2,2,2 --periodic 0,0,0 --agglomerate-below 65 --deep 1 --transport ipc --steps 20 --warmup 2 > gpurun_out/ts.log 2>&1 || { tail gpurun_out/ts.log; exit 1; }
f=$(find gpurun_out/ts -name "*kernel_trace.csv" | head -n 1)
python3 tools/trace_summary.py "$f" > gpurun_out/ts_split.txt
rm -rf gpurun_out/ts
head -45 gpurun_out/ts_split.txt
