#!/bin/bash
# A/B of the 8-GPU share proxy (tools/rank_proxy.py: 256^3, ipc self
# messages, deep halo), ROUNDS interleaved rounds over CONFIGS entries
# "lib:block:cap" -- lib "new" = the in-tree library, otherwise
# gpurun_ab/<lib>/libmgic.so; block = MGIC_IPC_BLOCK_ELEMS, cap =
# MGIC_IPC_GRID_CAP (0 = the library's default).  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=${OUT:-gpurun_out/proxy_ab.txt}
for r in $(seq ${ROUNDS:-2}); do
  for c in $CONFIGS; do
    IFS=: read -r v be cap <<< "$c"
    L=""; [ "$v" != new ] && L=gpurun_ab/$v/libmgic.so
    echo -n "$v block $be cap $cap " >> $out
    env MGIC_LIB_PATH=$L MGIC_IPC_BLOCK_ELEMS=$be MGIC_IPC_GRID_CAP=$cap \
      timeout -k 10 180 python3 tools/rank_proxy.py --transport ipc --deep 1 --steps ${STEPS:-30} \
      >> $out 2> gpurun_out/proxy_ab_err.log || { tail gpurun_out/proxy_ab_err.log; exit 1; }
  done
done
