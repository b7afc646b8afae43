#!/bin/bash
# round-4 GPU session g: the exchange launch's block size and grid cap on the
# 8-GPU share proxy (256^3, ipc self messages, deep halo): per config one
# rocprofv3 kernel trace (k_exchange lines) and two interleaved untraced runs
# (V-cycle time).  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
CONFIGS=${CONFIGS:-"4096:256 4096:1024 2048:1024 1024:1024 512:1024 1024:256"}
out=gpurun_out/exch_sweep.txt
: > $out
for c in $CONFIGS; do
  be=${c%%:*}; cap=${c##*:}
  MGIC_IPC_BLOCK_ELEMS=$be MGIC_IPC_GRID_CAP=$cap timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/xt" -o p --output-format csv -- python3 "$R/tools/rank_proxy.py" --transport ipc --deep 1 --steps 20 > gpurun_out/xt.log 2>&1 || { tail gpurun_out/xt.log; exit 1; }
  f=$(find gpurun_out/xt -name "*kernel_trace.csv" | head -n 1)
  echo "== block $be cap $cap" >> $out
  python3 tools/trace_summary.py "$f" | grep k_exchange >> $out
  rm -rf gpurun_out/xt
done
for r in 1 2; do
  for c in $CONFIGS; do
    be=${c%%:*}; cap=${c##*:}
    echo -n "block $be cap $cap " >> $out
    MGIC_IPC_BLOCK_ELEMS=$be MGIC_IPC_GRID_CAP=$cap timeout -k 10 180 python3 tools/rank_proxy.py --transport ipc --deep 1 --steps 30 >> $out 2> gpurun_out/xp_err.log || { tail gpurun_out/xp_err.log; exit 1; }
  done
done
cat $out
echo "session done"
