#!/bin/bash
# round-4 GPU session j: per-block flags in the exchange launch (each get
# block waits for its own put block) -- the GPU suite, then the 8-GPU share
# proxy A/B against prev (one atomic per block, whole-message waits) and cnt
# (per-workgroup counting, whole-message waits) over block sizes, and a
# kernel trace of the new library.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
: > gpurun_out/proxy_ab.txt
CONFIGS="prev:4096:0 cnt:4096:0 cnt:2048:0 new:4096:0 new:2048:0 new:1024:0" ROUNDS=2 bash tools/proxy_ab.sh || exit 1
python3 tools/proxy_ab_summary.py gpurun_out/proxy_ab.txt
for be in 4096 2048; do
  MGIC_IPC_BLOCK_ELEMS=$be timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/xt" -o p --output-format csv -- python3 "$R/tools/rank_proxy.py" --transport ipc --deep 1 --steps 20 > gpurun_out/xt.log 2>&1 || { tail gpurun_out/xt.log; exit 1; }
  f=$(find gpurun_out/xt -name "*kernel_trace.csv" | head -n 1)
  echo "== new block $be" >> gpurun_out/proxy_ab.txt
  python3 tools/trace_summary.py "$f" | grep "avg=" | grep k_exchange >> gpurun_out/proxy_ab.txt
  python3 tools/trace_summary.py "$f" > gpurun_out/ptrace_$be.txt
  rm -rf gpurun_out/xt
done
grep -A7 "^==" gpurun_out/proxy_ab.txt
echo "session done"
