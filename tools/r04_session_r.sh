#!/bin/bash
# round-4 GPU session r: exchange launch reads every peer's slot
# acknowledgement at kernel entry (one lane each) instead of the first put
# block's serial wait -- IPC / multi-process tests, then the 8-GPU share
# proxy A/B against prev, three interleaved rounds.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_multiprocess.py tests/test_gpu_parity.py tests/test_mixed.py -m gpu -q -x -rf -k "process or ipc or transport or multibox or eight or rccl or pipelined" --timeout 400 --timeout-method thread > gpurun_out/pytest_ipc.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_ipc.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_ipc.log; exit $rc; }
: > gpurun_out/proxy_ab.txt
CONFIGS="prev:0:0 new:0:0" ROUNDS=3 bash tools/proxy_ab.sh || exit 1
python3 tools/proxy_ab_summary.py gpurun_out/proxy_ab.txt
echo "session done"
