#!/bin/bash
# round-4 GPU session t: what the domain-face (edge) tiles cost the two-sweep
# launch -- kernel traces of a 512^3 and a 256^3 box, periodic in every
# direction (no edge tile) and with Dirichlet faces.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
: > gpurun_out/edge_cost.txt
for n in 512 256; do
  for per in 1,1,1 0,0,0; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/et" -o p --output-format csv -- python3 "$R/tools/rank_proxy.py" --size $n --local --deep 1 --periodic $per --steps 6 --warmup 1 > gpurun_out/et.log 2>&1 || { tail gpurun_out/et.log; exit 1; }
    f=$(find gpurun_out/et -name "*kernel_trace.csv" | head -n 1)
    echo "== n $n periodic $per" >> gpurun_out/edge_cost.txt
    python3 tools/trace_summary.py "$f" | grep "avg=" | grep -E "k_gsrb_tb2|k_residual|k_restrict|k_prolong" >> gpurun_out/edge_cost.txt
    rm -rf gpurun_out/et
  done
done
cat gpurun_out/edge_cost.txt
echo "session done"
