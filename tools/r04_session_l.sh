#!/bin/bash
# round-4 GPU session l: exchange grid cap x largest block x loads in flight
# per thread (u8: 8 instead of 4) on the 8-GPU share proxy.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/proxy_ab.txt
CONFIGS="new:2048:256 new:2048:512 new:4096:512 new:4096:768 u8:4096:512 u8:4096:256 u8:2048:512" ROUNDS=2 bash tools/proxy_ab.sh || exit 1
python3 tools/proxy_ab_summary.py gpurun_out/proxy_ab.txt
echo "session done"
