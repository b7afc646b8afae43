#!/bin/bash
# round-4 GPU session k: block size per item (16-32 blocks an item, capped)
# vs one block size (ff), and the exchange grid cap, on the 8-GPU share proxy;
# the IPC parity tests first.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_multiprocess.py tests/test_gpu_parity.py tests/test_mixed.py -m gpu -q -x -rf -k "process or ipc or transport or multibox or eight or rccl" --timeout 400 --timeout-method thread > gpurun_out/pytest_ipc.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_ipc.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_ipc.log; exit $rc; }
: > gpurun_out/proxy_ab.txt
CONFIGS="ff:2048:0 new:2048:0 new:4096:0 new:2048:512 new:2048:1024 cnt:2048:0" ROUNDS=2 bash tools/proxy_ab.sh || exit 1
python3 tools/proxy_ab_summary.py gpurun_out/proxy_ab.txt
MGIC_IPC_BLOCK_ELEMS=2048 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/xt" -o p --output-format csv -- python3 "$R/tools/rank_proxy.py" --transport ipc --deep 1 --steps 20 > gpurun_out/xt.log 2>&1 || { tail gpurun_out/xt.log; exit 1; }
f=$(find gpurun_out/xt -name "*kernel_trace.csv" | head -n 1)
python3 tools/trace_summary.py "$f" > gpurun_out/ptrace_k.txt
rm -rf gpurun_out/xt
grep "avg=" gpurun_out/ptrace_k.txt | grep k_exchange
echo "session done"
