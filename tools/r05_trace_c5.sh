#!/bin/bash
# rocprofv3 kernel trace of the mixed 1024^3 C5 bench (tools/bench_c5.py
# --kinds mixed, no oracle check) -> gpurun_out/tc5.txt.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/tc5" -o tc5 --output-format csv -- python3 "$R/tools/bench_c5.py" --kinds mixed --vcycles 4 --no-oracle-check > gpurun_out/tc5.log 2>&1 || { tail gpurun_out/tc5.log; exit 1; }
f=$(find gpurun_out/tc5 -name "*kernel_trace.csv" | head -n 1)
python3 tools/trace_summary.py "$f" > gpurun_out/tc5.txt
rm -rf gpurun_out/tc5
head -40 gpurun_out/tc5.txt
