#!/bin/bash
# round 5: the whole-split share proxy with the exchange's fixed cost taken
# as the device sees it (rank_proxy.py exchange_fixed_gpu_ms) beside the
# host-loop rate, three runs; then the split's kernel trace at HEAD.
# Measurement only; each step bounded.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/xg
: > gpurun_out/xg/proxy.txt
for i in 1 2 3; do
  timeout -k 10 200 python3 tools/rank_proxy.py --size 512 --parts 2,2,2 --periodic 0,0,0 --agglomerate-below 65 --deep 1 --transport ipc --steps 20 >> gpurun_out/xg/proxy.txt 2>> gpurun_out/xg/proxy_err.log || { tail gpurun_out/xg/proxy_err.log; exit 1; }
done
cat gpurun_out/xg/proxy.txt
if [ "${SKIP_TRACE:-0}" != 1 ]; then
  bash tools/r05_trace_split.sh || exit 1
  cp gpurun_out/ts_split.txt gpurun_out/xg/
fi
echo "xg session done"
