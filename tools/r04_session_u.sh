#!/bin/bash
# round-4 GPU session u: which faces the edge-tile cost comes from -- kernel
# traces of one 512^3 box periodic in x only, y only, x and y, z only.
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
: > gpurun_out/edge_faces.txt
for per in 1,0,0 0,1,0 1,1,0 0,0,1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/et" -o p --output-format csv -- python3 "$R/tools/rank_proxy.py" --size 512 --local --deep 1 --periodic $per --steps 6 --warmup 1 > gpurun_out/et.log 2>&1 || { tail gpurun_out/et.log; exit 1; }
  f=$(find gpurun_out/et -name "*kernel_trace.csv" | head -n 1)
  echo "== n 512 periodic $per" >> gpurun_out/edge_faces.txt
  python3 tools/trace_summary.py "$f" | grep "avg=" | grep -E "k_gsrb_tb2" >> gpurun_out/edge_faces.txt
  rm -rf gpurun_out/et
done
cat gpurun_out/edge_faces.txt
echo "session done"
